/*
 * subread_realign.h -- iteration two of the post-vote pipeline, host C:
 * the realignment that turns each read's vote records into CIGARs against the chunk's event
 * table, the choice among the read's (pair's) candidate alignments, and the SAM fields.
 *
 * It replaces do_iteration_two (reference src/core.c:2486-3018) and what it calls:
 *   explain_read           core-junction.c:2617-2777
 *   search_events_to_back  core-junction.c:588-746   (event jumps from the read tail)
 *   search_events_to_front core-junction.c:125-306   (event jumps towards the read tail)
 *   new_explain_try_replace core-junction.c:308-447  (best / tied explanations)
 *   finalise_explain_CIGAR core-junction.c:3159-3449 (CIGAR, event support lists)
 *   final_CIGAR_quality    core-junction.c:2899-3156 (soft clipping, mismatches)
 *   find_soft_clipping     core-junction.c:2820-2895
 *   write_realignments_for_fragment / convert_read_to_tmp / add_head_tail_cut_softclipping /
 *   calc_flags / calc_tlen / write_single_fragment   core.c:1367-1535,1635-1803,1888-2178,2383-2437
 *   test_PE_and_same_chro_align / calc_end_pos       core.c:4755-4815
 *   add_realignment_event_support                    core.c:2364-2379
 * with the event site lists as iteration two sees them: sort_junction_entry_table
 * (core-indel.c:847-929, at most MAX_EVENT_ENTRIES_PER_SITE = 9 per coordinate, ordered by
 * scanning_events_compare) minus what remove_neighbour took out (core-indel.c:573-593).
 *
 * Covered: base-space reads (FASTQ or FASTA), SAM fields, subread-align (-t 0 / -t 1) and
 * subjunc defaults and their realignment options (-M, --multiMapping, -B, --keepReadOrder
 * order, --ignoreUnmapped, --rg, --maxMismatches, --minFragLength/--maxFragLength, -S,
 * --noTLENpreference, --complexIndels, --min_mapped_fraction, -P 6).
 * Not covered (svg_realign_create returns SVG_E_UNSUPPORTED; a caller keeps the reference's own
 * iteration two for them): colour space, fusion / long-deletion detection (strand-jumped
 * sections, chimeric CIGARs), the annotation's exonic-region bitmap (-a with exon scoring),
 * scRNA mode, big-margin read filtering (do_big_margin_filtering_for_reads).
 *
 * Threading: svg_realign_chunk runs its own worker threads; the fragments come out through an
 * svg_sam_writer (subread_sam.h) in fragment order, or through a callback in fragment order.
 */
#ifndef SUBREAD_REALIGN_H
#define SUBREAD_REALIGN_H

#include <stdint.h>
#include "subread_vote.h"
#include "subread_events.h"
#include "subread_sam.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SVG_EXPERIMENT_DNASEQ 1000   /* CORE_EXPERIMENT_DNASEQ, core.h:278 */
#define SVG_EXPERIMENT_RNASEQ 2000   /* CORE_EXPERIMENT_RNASEQ */

/* the configuration fields iteration two reads (configuration_t, core.h) */
typedef struct svg_realign_params {
	int32_t paired;                         /* input_reads.is_paired_end_reads                    */
	int32_t multi_best;                     /* config.multi_best_reads: records per read end      */
	int32_t reported_multi_best;            /* config.reported_multi_best_reads (-B)              */
	int32_t report_multi_mapping;           /* config.report_multi_mapping_reads (--multiMapping) */
	int32_t min_votes_first;                /* config.minimum_subread_for_first_read (-m)         */
	int32_t min_votes_second;               /* config.minimum_subread_for_second_read (-p)        */
	int32_t experiment_type;                /* SVG_EXPERIMENT_* (-t; subjunc: RNA)                */
	int32_t max_mismatch_exonic;            /* config.max_mismatch_exonic_reads (-M)              */
	int32_t max_mismatch_junction;          /* config.max_mismatch_junction_reads                 */
	int32_t min_mapped_fraction;            /* config.min_mapped_fraction                         */
	int32_t show_soft_clipping;             /* config.show_soft_cliping                           */
	int32_t realignment_minimum_variant_distance;
	int32_t limited_tree_scan;
	int32_t maximise_sensitivity_indel;     /* --complexIndels                                    */
	float   minimum_exonic_subread_fraction;
	int32_t no_tlen_preference;             /* --noTLENpreference                                 */
	int32_t min_pair_distance, max_pair_distance;
	int32_t is_first_read_reversed, is_second_read_reversed;
	int32_t do_breakpoint_detection;        /* subjunc: XS:A tags                                 */
	int32_t ignore_unmapped_reads;          /* --ignoreUnmapped                                   */
	int32_t phred_offset;                   /* 33 (FASTQ_PHRED33) or 64 (-P 6)                    */
	char    read_group_id[320];             /* --rg ("" = none; the tag is cut at 310 bytes)      */
	/* unsupported configurations (must be 0) */
	int32_t do_fusion_detection, do_long_del_detection, color_space, exonic_region_bitmap,
	        scrna_input_mode, do_big_margin_filtering_for_reads;
} svg_realign_params;

/* the reference's defaults after the program's own option parsing with no options:
 * program SVG_PROGRAM_ALIGN (-t 1 DNA unless rna) or SVG_PROGRAM_SUBJUNC */
void svg_realign_params_default(svg_realign_params *p, int program, int paired, int rna);

/* the chunk's reads as fetch_next_read_pair hands them to iteration two (-S reversal applied):
 * read i, end e: name at buf + name_off[i*ends+e], text at buf + text_off[...] (len[...] bytes),
 * quality at buf + qual_off[...] ("" = none, as FASTA input); strings NUL-terminated */
typedef struct svg_fragment_reads {
	const char *buf;
	const uint64_t *name_off, *text_off, *qual_off;
	const uint16_t *len;
	uint64_t n;                             /* fragments (reads or pairs) */
} svg_fragment_reads;

/* the counters write_realignments_for_fragment / calc_flags / write_single_fragment add to
 * (thread_context_t fields summed by run_maybe_threads, core.c:3433-3444) */
typedef struct svg_realign_stats {
	int64_t all_mapped_reads, all_correct_PE_reads, not_properly_pairs_wrong_arrangement,
	        not_properly_pairs_different_chro, not_properly_different_strands, not_properly_pairs_TLEN_wrong,
	        all_unmapped_reads, not_properly_pairs_only_one_end_mapped, all_multimapping_reads,
	        all_uniquely_mapped_reads;
} svg_realign_stats;

/* the per-fragment output hook when no svg_sam_writer is given: called in fragment order (one
 * caller at a time) for every location, with the two records of a pair (rec2 NULL for single
 * end).  fragment = chunk read number, this_location of all_locations. */
typedef void (*svg_realign_emit_fn)(void *arg, int64_t fragment, int all_locations, int this_location,
                                    const svg_sam_record *rec1, const svg_sam_record *rec2);

typedef struct svg_realign svg_realign;

int  svg_realign_create(const svg_genome_arrays *g, const svg_realign_params *p, svg_realign **out);
void svg_realign_destroy(svg_realign *ra);

/*
 * The chunk's event table as iteration two sees it: the merged table after the anti-supporting
 * read scan and remove_neighbour (svg_events_get of a table after svg_events_remove_neighbour;
 * events with event_type 0 are the ones remove_neighbour removed in this chunk).  The site lists
 * are built the way sort_junction_entry_table builds them, before the removals.
 * final_counted_reads / junction_flanking_* of the copy are what the chunk's realignment adds.
 */
int svg_realign_set_events(svg_realign *ra, const svg_event *ev, int64_t n);
/* the events with this chunk's realignment support added (n = the count given above) */
int svg_realign_get_events(const svg_realign *ra, svg_event *out);

/* expected-TLEN state across chunks (global_context_t.expected_TLEN_read_numbers / _sum) */
void svg_realign_set_tlen_state(svg_realign *ra, int64_t read_numbers, int64_t sum);
void svg_realign_get_tlen_state(const svg_realign *ra, int64_t *read_numbers, int64_t *sum);

/*
 * Iteration two over one chunk: `records` is the bigtable of the chunk (n x ends x multi_best
 * mapping_result_t, as the vote and the event stage left them; updated as the reference updates
 * them: selected_votes of filtered records, result_flags CORE_IS_FULLY_EXPLAINED, read_length,
 * selected_position + soft clipping of written records).  SAM goes to `sink` (after
 * svg_sam_writer_begin_chunk(sink, n) by the caller) or, when sink is NULL, to `emit`.
 * `stats` (may be NULL) is added to.  threads <= 0: the library's host thread count.
 */
int svg_realign_chunk(svg_realign *ra, const svg_fragment_reads *reads, svg_mapping_result *records,
                      svg_sam_writer *sink, svg_realign_emit_fn emit, void *emit_arg, int threads,
                      svg_realign_stats *stats);

/* contig table of a genome image (for SAM headers): n, names and lengths as write_sam_headers
 * prints them in @SQ LN (FETCH_SEQ_LEN, core.c:3841: read_offsets delta + 16 - 2 * padding) */
int svg_genome_arrays_contigs(const svg_genome_arrays *g, uint32_t *n, const char **names, uint32_t *lengths);

/*
 * A genome image over memory the caller keeps alive (e.g. the reference's own
 * gene_value_index_t arrays and gene_offset_t table inside a drop-in): no file is read and the
 * value arrays are not copied.  blocks[b] = {values, start_point, length, start_base_offset,
 * values_bytes} as gvindex_load leaves them; names: n_chr strings of name_stride bytes.
 */
typedef struct svg_value_block {
	const uint8_t *values;
	uint32_t start_point, length, start_base_offset, values_bytes;
} svg_value_block;
int svg_genome_arrays_wrap(const svg_value_block *blocks, int nblocks, const uint32_t *chr_end, const char *names,
                           int name_stride, uint32_t n_chr, int padding, int gap, svg_genome_arrays **out);

#ifdef __cplusplus
}
#endif
#endif
