/*
 * subread_sam.h -- SAM emission for the post-vote pipeline, host C.
 *
 * In the reference, iteration two (do_iteration_two, core.c:2486-3018) runs on -T threads and
 * every thread hands its fragment's finished SAM lines to add_buffered_fragment
 * (core.c:1835-1884), which writes them in fragment order: under the global output lock a
 * thread writes only when last_written_fragment_number == its fragment - 1, and otherwise
 * releases the lock, sleeps (usleep(2)) and tries again.  With SAM output every thread of the
 * step takes its turn through that spin, one fragment at a time.
 *
 * svg_sam_writer keeps the output identical -- the same lines, in fragment order, each
 * fragment's locations in the order they are put -- without any thread waiting for another:
 * a put stores its text in a reorder ring keyed by the fragment number, and whichever thread
 * completes the oldest missing fragment writes every fragment that is complete from there on,
 * batched into large writes.  svg_sam_format builds one SAM line exactly as the reference's
 * format string does ("%s\t%d\t%s\t%u\t%d\t%s\t%s\t%u\t%d\t%s\t%s%s%s\n", core.c:1865-1867),
 * without stdio.
 *
 * Conventions as in subread_vote.h: 0 or a negative SVG_E_* code, svg_last_error() for text.
 */
#ifndef SUBREAD_SAM_H
#define SUBREAD_SAM_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct svg_sam_writer svg_sam_writer;

/* `file` is the FILE* the SAM header went to (output_sam_fp, core.c:3870-3887); the writer
 * appends to it with fwrite after the caller's own writes, and fflush()es it on close. */
int  svg_sam_writer_open(void *file, svg_sam_writer **out);
/* every fragment put so far is written; then the writer is freed (the FILE* stays open) */
int  svg_sam_writer_close(svg_sam_writer *w);
/* a new read chunk of n_fragments fragments: fragment numbers start again at 0
 * (run_maybe_threads resets last_written_fragment_number to -1 before each iteration two,
 * core.c:3384-3386); the chunk's text is flushed to the FILE* as soon as its last fragment is
 * written.  Returns SVG_E_ARG if fragments of the previous chunk are still missing. */
int  svg_sam_writer_begin_chunk(svg_sam_writer *w, int64_t n_fragments);
/* fragment `fragment` (0-based in the chunk), location `location` of `all_locations`: its text
 * (one or two SAM lines) is written after every earlier fragment and every earlier location of
 * this fragment.  Thread-safe; never waits for other producers. */
int  svg_sam_writer_put(svg_sam_writer *w, int64_t fragment, int location, int all_locations,
                        const char *text, size_t len);
/* the complete text of `count` consecutive fragments first .. first+count-1 (all their
 * locations, in order) in one put: the same as putting each fragment whole, with one lock
 * round trip.  A producer that owns a run of fragments (svg_realign_chunk's workers take blocks
 * of them) puts the run this way.  Empty text is allowed (fragments that write nothing). */
int  svg_sam_writer_put_block(svg_sam_writer *w, int64_t first, int64_t count, const char *text, size_t len);
/*
 * BAM output (the reference's default; SamBam_writer_add_read, sambam-file.c:1704-1797): the same
 * ordered sink over binary records.  `file` is the BAM file's FILE* after the writer that made it
 * wrote the header blocks (SamBam_writer_finish_header, core.c:3870); `paired`: two records per
 * location (the pair), else one; `level`: the deflate level (the reference's Z_BEST_SPEED, 1).
 * Producers put svg_bam_format records -- per location the record of each end, locations in order.
 * The records leave as BGZF blocks cut where the reference's single ordered stream cuts them
 * (after a location that takes the block past 55000 bytes), each deflated by the thread that cut
 * it; a partial block carries over to the next chunk and is written by svg_sam_writer_close, which
 * does not write the BAM end-of-file block (the BAM writer that owns the file does, when it closes).
 */
int  svg_sam_writer_open_bam(void *file, int paired, int level, svg_sam_writer **out);
int  svg_sam_writer_is_bam(const svg_sam_writer *w);
/* fragments put but not yet written (waiting for an earlier one) */
int64_t svg_sam_writer_pending(svg_sam_writer *w);
/* 1 once a write came up short (the reference's output_sam_is_full, core.c:1869-1871) */
int  svg_sam_writer_failed(svg_sam_writer *w);

/* one SAM record as write_single_fragment hands it to add_buffered_fragment (core.c:2125-2131) */
typedef struct svg_sam_record {
	const char *qname;
	int32_t     flag;
	const char *rname;
	uint32_t    pos;
	int32_t     mapq;
	const char *cigar;
	const char *rnext;
	uint32_t    pnext;
	int32_t     tlen;
	const char *seq;
	const char *qual;
	const char *tags;      /* without the leading tab; "" = none */
} svg_sam_record;

/* Appends the record's line to buf (cap bytes); returns its length, or a negative SVG_E_ARG when
 * it does not fit (nothing is guaranteed about buf then). */
int64_t svg_sam_format(const svg_sam_record *r, char *buf, size_t cap);

/* The record in BAM binary form, byte for byte as SamBam_writer_add_read builds it from the same
 * fields (block size, refID, pos - 1, bin / MAPQ / name length, flag / CIGAR op count, l_seq,
 * next refID, pnext - 1, tlen, name, CIGAR ops, 4-bit bases, qualities - 33, tags as
 * SamBam_compress_additional encodes them).  refid / next_refid: the contigs' indexes in the BAM
 * header (the index's contig order; -1 for '*'); read_len: l_seq, the read's length (the text
 * and quality hold that many bytes).  One difference: a text with a NUL byte inside encodes up to
 * the NUL, as the reference's does, and the rest of its 4-bit field is zero here where the
 * reference's record carries whatever its stream buffer held at that place.  Returns the bytes
 * written, or SVG_E_ARG when cap is too small. */
int64_t svg_bam_format(const svg_sam_record *r, int32_t refid, int32_t next_refid, int32_t read_len, char *buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif /* SUBREAD_SAM_H */
