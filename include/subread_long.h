/*
 * subread_long.h -- C ABI of sublong's voting step on the MI355X (long reads: ONT / PacBio).
 *
 * sublong (src/longread-one) maps each read in two stages per read
 * (LRMchunk_read_iteration, longread-mapping.c:1343-1348):
 *   LRMdo_one_voting_read         longread-mapping.c:552-560
 *       both strands (strand 1 = LRMreverse_read of the read, LRMfile-io.c:71), subreads every
 *       ~3 bases (LRMcalc_total_subreads / LRMcalc_subread_start, longread-mapping.c:516-538),
 *       each probed with LRMgehash_go_QQ (LRMsorted-hashtable.c:443-518) into a 64973-row x
 *       51-slot vote table: a hit votes for the slot holding exactly its position on the same
 *       strand while it is within 14 bases of the slot's coverage end, or opens a new slot
 *   LRMdo_dynamic_programming_read longread-mapping.c:1314-1334
 *       starts with LRMcopy_longvotes_to_itr (:668-682, the table row-major) and LRMmerge_sort by
 *       position + coverage start (:1317, LRMhelper.c:26-43); windows, chains and gap filling
 *       follow on the host.
 * svg_long_vote_batch replaces the voting stage and that copy + sort for a batch of reads: its
 * output is the vote table's slots in LRMcopy_longvotes_to_itr's order and the permutation
 * LRMmerge_sort leaves, so the host continues at LRMfind_top_windows (longread-mapping.c:1321)
 * with the reference's own arrays.  The index is block 0 of a Subread index (LRMload_index,
 * longread-mapping.c:377-388), opened with svg_index_open.
 *
 * Conventions as in subread_vote.h: 0 or a negative SVG_E_* code, svg_last_error() for the text.
 */
#ifndef SUBREAD_LONG_H
#define SUBREAD_LONG_H

#include "subread_vote.h"

#ifdef __cplusplus
extern "C" {
#endif

/* reference constants (LRMconfig.h:26-28,47,67-68) */
#define SVG_LONG_MAX_READ_LENGTH   1200000          /* LRMMAX_READ_LENGTH */
#define SVG_LONG_READ_KEEP         (SVG_LONG_MAX_READ_LENGTH - 1)   /* LRMgeinput_readline keeps 1199999 */
#define SVG_LONG_VOTE_TABLE_SIZE   64973            /* LRMGENE_VOTE_TABLE_SIZE */
#define SVG_LONG_VOTE_SPACE        51               /* LRMGENE_VOTE_SPACE */
#define SVG_LONG_NEGATIVE_STRAND   4                /* LRMIS_NEGATIVE_STRAND */

/* Reads as LRMfetch_next_read hands them to LRMdo_one_voting_read: ASCII text (read_text, the
 * forward strand as read from the file), lengths up to SVG_LONG_READ_KEEP. */
typedef struct svg_long_reads {
	const char     *seq;
	const uint64_t *offsets;
	const uint32_t *lens;
	uint64_t        n_reads;
} svg_long_reads;

/* One used slot of the read's LRMgene_vote_t (LRMconfig.h:75-86) -- the fields the host stages
 * read: pos, votes, masks (strand), coverage_start / coverage_end. */
typedef struct svg_long_vote {
	uint32_t pos;              /* vote_table.pos[bb][ii]: chromosome position minus subread offset */
	uint32_t coverage_start;   /* first voting subread's offset in the (strand's) read */
	uint32_t coverage_end;     /* last voting subread's offset + 16 */
	uint16_t votes;            /* unsigned short, as the reference counts (wraps past 65535) */
	uint8_t  negative;         /* masks[bb][ii] & LRMIS_NEGATIVE_STRAND ? 1 : 0 */
	uint8_t  _pad;
	uint32_t slot;             /* bb << 16 | ii (sorting_subread_nos) */
} svg_long_vote;

typedef struct svg_long_result {
	uint64_t       n_reads;
	uint64_t      *vstart;     /* n_reads + 1: read r's slots are votes[vstart[r] .. vstart[r+1]) */
	svg_long_vote *votes;      /* per read, row-major (bb, ii): LRMcopy_longvotes_to_itr's order */
	uint32_t      *order;      /* per read, aligned with votes: order[vstart[r] + k] = the index
	                              (within the read) of the slot LRMmerge_sort puts at position k
	                              (key pos + coverage_start, u32) */
} svg_long_result;

/* The voting stage of a batch (host buffers, synchronous); result arrays are owned by the
 * library until svg_long_free.  Reads longer than SVG_LONG_READ_KEEP: SVG_E_ARG. */
int  svg_long_vote_batch(svg_index *idx, const svg_long_reads *reads, svg_long_result *out);
void svg_long_free(svg_long_result *r);

#ifdef __cplusplus
}
#endif
#endif
