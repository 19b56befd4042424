/*
 * subread_events.h -- host-side event detection on the vote records: the tail of the
 * reference's final voting run (do_voting, core.c:3241-3290), which turns each read's
 * mapping records into indel and junction events of a chromosome event table, and the
 * per-thread table merge that follows the voting step (finalise_indel_and_junction_thread,
 * core-indel.c:1012-1141).  This is the first stage of the host post-vote pipeline
 * (SURVEY.md §8(f) row 2); it consumes svg_vote_batch's records unchanged and marks them
 * CORE_IS_GAPPED_READ (flag 64) exactly where the reference does (mark_gapped_read,
 * core.h:61).
 *
 * Covered (the configuration subread-align and subjunc run by default):
 *   find_new_indels   core-indel.c:1831-2098, dynamic-programming path
 *                     (use_dynamic_programming_indel = 1, core-interface-aligner.c:271,
 *                     core-interface-subjunc.c:270; core_dynamic_align core-indel.c:4573)
 *   find_new_junctions core-junction.c:3836-4137 (do_breakpoint_detection), with
 *                     core_search_short_exons (core-junction.c:4386-4731) for reads > 160 bp
 *   the events of fragile junction voting (core-junction.c:5211-5419) for subjunc reads
 *                     > 160 bp, from svg_fragile_batch's windows (svg_events_add_batch2)
 *   local_add_indel_event / put_new_event / search_event  core-indel.c:1385-1569
 *   has_better_mapping core.c:3035, is_ambiguous_voting core-junction.c:3522,
 *   locate_current_value_index core.c:2216 (multi-block indexes)
 *   anti_supporting_read_scan core-indel.c:177-330
 * Not covered (SVG_E_UNSUPPORTED): fusion / long-deletion detection, the extending indel
 * search (extending_search_indels = 0 in both programs).
 *
 * Threading: one table per host thread; svg_events_merge() combines tables the way
 * finalise_indel_and_junction_thread combines the reference's per-thread tables.
 */
#ifndef SUBREAD_EVENTS_H
#define SUBREAD_EVENTS_H

#include <stdint.h>
#include "subread_vote.h"

#ifdef __cplusplus
extern "C" {
#endif

/* event_type values (core-indel.h:35-41) */
#define SVG_EVENT_INDEL     8
#define SVG_EVENT_JUNCTION 64
#define SVG_EVENT_FUSION  128

/* one chromosome_event_t (core.h:274-346) with the inserted bases decoded */
typedef struct svg_event {
	uint32_t small_side;                  /* event_small_side (linear, padded coordinates) */
	uint32_t large_side;                  /* event_large_side                               */
	int16_t  indel_length;                /* >0 deletion, <0 insertion, 0 junction          */
	int16_t  junction_flanking_left;
	int16_t  junction_flanking_right;
	int8_t   indel_at_junction;
	int8_t   is_negative_strand;
	int8_t   is_strand_jumped;
	int8_t   is_donor_found_or_annotation;
	int8_t   small_side_increasing_coordinate;
	int8_t   large_side_increasing_coordinate;
	int8_t   connected_next_event_distance;
	int8_t   connected_previous_event_distance;
	uint16_t supporting_reads;
	uint16_t anti_supporting_reads;
	uint16_t final_counted_reads;
	uint16_t final_reads_mismatches;
	uint8_t  event_type;                  /* SVG_EVENT_*                                    */
	uint8_t  inserted_len;                /* bases in inserted_bases (insertions)           */
	uint64_t critical_read_id;            /* 2 * read number + end, junctions               */
	float    event_quality;
	int32_t  critical_supporting_reads;
	char     inserted_bases[40];          /* ACGT text of an insertion (not terminated)     */
} svg_event;

/* knobs of the event search with the reference's defaults (core-indel.c:4512-4515) */
typedef struct svg_event_params {
	int32_t dp_penalty_create_gap;        /* -1 */
	int32_t dp_penalty_extend_gap;        /*  0 */
	int32_t dp_match_score;               /*  2 */
	int32_t dp_mismatch_penalty;          /*  0 */
	int32_t report_multi_mapping_reads;   /*  0 (--multiMapping: 1) */
	int32_t quality_base;                 /* '#' (35): FASTQ_PHRED33; 'B' (66) with -P 6 (read_quality_score) */
	int32_t maximise_sensitivity_indel;   /*  0 (the fragile votes' indels: < 2 mismatches, else <= 2) */
} svg_event_params;
void svg_event_params_default(svg_event_params *e);

/* host copy of the index's base arrays (every <prefix>.NN.b.array) and contig table */
typedef struct svg_genome_arrays svg_genome_arrays;
int  svg_genome_arrays_open(const char *prefix, svg_genome_arrays **out);
void svg_genome_arrays_close(svg_genome_arrays *g);

typedef struct svg_events svg_events;
int  svg_events_create(svg_events **out);
void svg_events_destroy(svg_events *t);

/*
 * Add the events of a batch of voted reads (read i of the batch is read number
 * first_read + i of the reference's chunk numbering).  r1/r2/params are those given to
 * the vote; out/jout/big_margin are its records (jout / big_margin as the vote required
 * them).  Reads are processed in order, ends R1 then R2, records best 0..multi_best-1,
 * like do_voting.  out's result_flags gain CORE_IS_GAPPED_READ where the reference sets it.
 */
int svg_events_add_batch(svg_events *t, const svg_genome_arrays *g, const svg_params *p, const svg_event_params *ep,
                         const svg_reads *r1, const svg_reads *r2, uint64_t first_read, svg_mapping_result *out,
                         const svg_subjunc_result *jout, const uint16_t *big_margin);

/*
 * The same with what subjunc reads longer than 160 bases need as well (svg_events_add_batch
 * refuses those with SVG_E_UNSUPPORTED):
 *   q1 / q2 : the reads' quality strings (same offsets and lengths as r1 / r2; NULL = no
 *             qualities, as FASTA input) -- core_search_short_exons tests the head / tail quality;
 *   frag    : svg_fragile_batch's result for the same reads and parameters.
 * The events come in the reference's order: the fragile windows of every index block but the
 * last (the earlier runs of the block loop, core.c:3567-3613), then read by read the last
 * block's windows of the read followed by its final-run tail.
 */
int svg_events_add_batch2(svg_events *t, const svg_genome_arrays *g, const svg_params *p, const svg_event_params *ep,
                          const svg_reads *r1, const svg_reads *r2, const svg_reads *q1, const svg_reads *q2,
                          uint64_t first_read, svg_mapping_result *out, const svg_subjunc_result *jout,
                          const uint16_t *big_margin, const svg_fragile_result *frag);

/*
 * The events of the fragile junction-voting windows of ONE index block -- what a run of the
 * reference's block loop other than the last adds (core_fragile_junction_voting in do_voting,
 * core.c:3138-3142, for every read of the chunk; core-junction.c:5211-5419): every window of
 * `frag` (all of block `block`, reads of this batch), in order.  The final run's part is
 * svg_events_add_batch2's (given only the last block's windows).
 */
int svg_events_add_windows(svg_events *t, const svg_genome_arrays *g, const svg_params *p, const svg_event_params *ep,
                           const svg_reads *r1, const svg_reads *r2, const svg_fragile_result *frag, int block);

/* Merge `n` tables (in order) into `dst` (created empty by the caller): the sort-and-sum of
 * finalise_indel_and_junction_thread.  Also call it with n = 1 on a single table: the merged
 * table is sorted by (small side, large side, indel length) as the reference's is. */
int svg_events_merge(svg_events *dst, svg_events *const *tables, int n);

/*
 * anti_supporting_read_scan (core-indel.c:177-330) on a merged table: every record of the
 * batch (n_reads x ends x multi_best, as the vote wrote them) that covers an event's side
 * strictly inside its covered range (5 bases in from both ends) counts one anti-supporting
 * read for it.  Run it once per chunk after svg_events_merge, as the reference does after
 * its voting step.
 */
int svg_events_anti_support(svg_events *t, const svg_params *p, const svg_event_params *ep, uint64_t n_reads, int ends,
                            const svg_mapping_result *out);

/*
 * remove_neighbour (core-indel.c:447-595) on a merged table after svg_events_anti_support, as
 * the reference runs it before iteration two (core.c:3629-3630): redundant neighbour events
 * become type 0 (CHRO_EVENT_TYPE_REMOVED) and leave the table's site lists.  Events of earlier
 * passes already removed stay removed.
 */
int svg_events_remove_neighbour(svg_events *t);

/* Append n events (e.g. a table kept from an earlier chunk, or the reference's own table) to t,
 * each entered in its sides' site lists in order as put_new_event does (core-indel.c:1385). */
int svg_events_load(svg_events *t, const svg_event *ev, int64_t n);

/*
 * Append n events exactly as a host's own event table holds them: the events (event ids in t
 * continue from its current count) WITHOUT entering them in site lists, then the site lists as
 * given -- list s is coordinate pos[s]'s, with entries ids[s * 9 .. s * 9 + cap[s] - 1] (event id
 * + 1 within ev, 0 ends the list) and room for cap[s] entries (1..9).  This is the state of the
 * reference's event_entry_table whatever made it: put_new_event's lists (room 9, a put keeps a 0
 * after the last entry), sort_junction_entry_table's (room = entries, core-indel.c:897-906, so no
 * put fits), remove_neighbour's compactions (core-indel.c:573-593).  The event searches and puts of
 * svg_events_add_batch2 / svg_events_add_windows then see the lists the reference's would.
 */
int svg_events_load_sites(svg_events *t, const svg_event *ev, int64_t n, const uint32_t *pos, const uint32_t *ids,
                          const uint8_t *cap, int64_t n_sites);

int64_t svg_events_count(const svg_events *t);
int     svg_events_get(const svg_events *t, svg_event *out);   /* svg_events_count() entries */

#ifdef __cplusplus
}
#endif
#endif
