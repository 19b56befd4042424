/*
 * TEST INFRASTRUCTURE ONLY -- never linked into the product.
 *
 * Vote-record dump hook for the REFERENCE aligner (oracle/_ref).  It is linked
 * into subread-align / subjunc built from the untouched reference sources under
 * /root/reference/src (see oracle/Makefile) with
 *     -Wl,--wrap=anti_supporting_read_scan
 * so that the call made by read_chunk_circles() right after the voting step of
 * every read chunk (/root/reference/src/core.c:3629) first lands here.  At that
 * point the bigtable holds the final post-vote mapping_result_t[multi_best] of
 * every read end of the chunk (core-bigtable.c:84-131).  The only field the
 * tail of do_voting (find_new_indels / find_new_junctions, core.c:3241-3290)
 * changes is result_flags bit CORE_IS_GAPPED_READ (64), through
 * mark_gapped_read (core.h:61; core-indel.c:1979,2089,2210,2220;
 * core-junction.c:3980); the voting step itself never sets that bit.  The dump
 * therefore clears bit 64, which makes the bytes identical to a dump taken
 * right after the strand loop of do_voting (core.c:3237)
 * -- the boundary the GPU path replaces.
 *
 * Output (env SVG_REF_DUMP=<file>, appended chunk after chunk, read order):
 *   for each read (pair) of the chunk:
 *     for end in {R1[,R2]}: for best in 0..multi_best-1: raw mapping_result_t (68 B)
 *     if do_breakpoint_detection:
 *       for end: for best: raw subjunc_result_t (16 B)
 *     if do_big_margin_filtering_for_junctions:
 *       for end: raw big-margin record (unsigned short[big_margin_record_size=9])
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "subread.h"
#include "core.h"
#include "core-bigtable.h"
#include "core-indel.h"

/*
 * Event-table dump (env SVG_REF_EVENTS=<file>, appended chunk after chunk): the indel /
 * junction event table of the final voting run as finalise_indel_and_junction_thread left
 * it (core-indel.c:1012-1141; run the aligner with -T 1 so that every event comes from one
 * thread table in read order) and anti_supporting_read_scan then counted (core-indel.c:268),
 * then the raw result_flags (CORE_IS_GAPPED_READ included) of every mapping record, in the
 * record order of the vote dump.
 *   u64 n_events, then n_events x svg_ref_event (96 B, layout below),
 *   u64 n_records, then n_records x u16 result_flags
 */
typedef struct {
	unsigned int small_side, large_side;
	short indel_length, junction_flanking_left, junction_flanking_right;
	char indel_at_junction, is_negative_strand, is_strand_jumped, is_donor_found_or_annotation;
	char small_side_increasing_coordinate, large_side_increasing_coordinate;
	char connected_next_event_distance, connected_previous_event_distance;
	unsigned short supporting_reads, anti_supporting_reads, final_counted_reads, final_reads_mismatches;
	unsigned char event_type, inserted_len;
	unsigned long long critical_read_id;
	float event_quality;
	int critical_supporting_reads;
	char inserted_bases[40];
} svg_ref_event;

void get_insertion_sequence(global_context_t *global_context, thread_context_t *thread_context, char *binary_bases,
                            char *read_text, int insertions);

static void dump_events(global_context_t *gc, const char *fn)
{
	FILE *fp = fopen(fn, "ab");
	if (!fp) return;
	indel_context_t *ic = (indel_context_t *)gc->module_contexts[MODULE_INDEL_ID];
	unsigned long long n = ic ? ic->total_events : 0, i, nrec;
	fwrite(&n, 8, 1, fp);
	for (i = 0; i < n; i++) {
		chromosome_event_t *e = ic->event_space_dynamic + i;
		svg_ref_event o;
		memset(&o, 0, sizeof o);
		o.small_side = e->event_small_side; o.large_side = e->event_large_side;
		o.indel_length = e->indel_length;
		o.junction_flanking_left = e->junction_flanking_left; o.junction_flanking_right = e->junction_flanking_right;
		o.indel_at_junction = e->indel_at_junction; o.is_negative_strand = e->is_negative_strand;
		o.is_strand_jumped = e->is_strand_jumped; o.is_donor_found_or_annotation = e->is_donor_found_or_annotation;
		o.small_side_increasing_coordinate = e->small_side_increasing_coordinate;
		o.large_side_increasing_coordinate = e->large_side_increasing_coordinate;
		o.connected_next_event_distance = e->connected_next_event_distance;
		o.connected_previous_event_distance = e->connected_previous_event_distance;
		o.supporting_reads = e->supporting_reads; o.anti_supporting_reads = e->anti_supporting_reads;
		o.final_counted_reads = e->final_counted_reads; o.final_reads_mismatches = e->final_reads_mismatches;
		o.event_type = e->event_type;
		o.critical_read_id = e->critical_read_id;
		o.event_quality = e->event_quality;
		o.critical_supporting_reads = e->critical_supporting_reads;
		if (e->event_type == CHRO_EVENT_TYPE_INDEL && e->indel_length < 0 && e->inserted_bases) {
			char buf[MAX_INSERTION_LENGTH + 2];
			int k = -e->indel_length;
			get_insertion_sequence(gc, NULL, e->inserted_bases, buf, k);
			if (k > (int)sizeof o.inserted_bases) k = sizeof o.inserted_bases;
			memcpy(o.inserted_bases, buf, k);
			o.inserted_len = (unsigned char)k;
		}
		fwrite(&o, sizeof o, 1, fp);
	}
	{
		long long r, nr = gc->processed_reads_in_chunk;
		int ends = 1 + gc->input_reads.is_paired_end_reads, mb = gc->config.multi_best_reads, e, b;
		nrec = (unsigned long long)nr * ends * mb;
		fwrite(&nrec, 8, 1, fp);
		for (r = 0; r < nr; r++)
			for (e = 0; e < ends; e++)
				for (b = 0; b < mb; b++) {
					unsigned short f = (unsigned short)_global_retrieve_alignment_ptr(gc, r, e, b)->result_flags;
					fwrite(&f, 2, 1, fp);
				}
	}
	fclose(fp);
}

int __real_anti_supporting_read_scan(global_context_t *global_context);
void __real_remove_neighbour(global_context_t *global_context);

/* SVG_REF_EVENTS_RN=<file>: the event types after remove_neighbour (core-indel.c:447, called
 * right after anti_supporting_read_scan, core.c:3629-3630; removed events become type 0),
 * appended chunk after chunk: u64 n_events, then n_events x u8 event_type */
void __wrap_remove_neighbour(global_context_t *gc)
{
	__real_remove_neighbour(gc);
	const char *fn = getenv("SVG_REF_EVENTS_RN");
	if (!fn || !fn[0]) return;
	FILE *fp = fopen(fn, "ab");
	if (!fp) return;
	indel_context_t *ic = (indel_context_t *)gc->module_contexts[MODULE_INDEL_ID];
	unsigned long long n = ic ? ic->total_events : 0, i;
	fwrite(&n, 8, 1, fp);
	for (i = 0; i < n; i++) {
		unsigned char t = (unsigned char)ic->event_space_dynamic[i].event_type;
		fwrite(&t, 1, 1, fp);
	}
	fclose(fp);
}
int __real_write_indel_final_results(global_context_t *global_context);

/* SVG_REF_TIMING=1: the reference's own phase clocks, accumulated over every chunk by
 * read_chunk_circles (core.c:3552-3641) -- index loading, the voting step, the stage between
 * voting and realignment (anti_supporting_read_scan + remove_neighbour + rewind, core.c:3613-3634)
 * and iteration two (realignment + SAM writing, core.c:3636-3641).  The reference's own print
 * of them is commented out (core.c:480-485).  write_final_results calls
 * write_indel_final_results (core.c:1220) once, after the last chunk, so the clocks are final
 * here; the wall clock of the whole run so far (start_time, core.c:4013) is printed beside them. */
/* the drop-in's ordered SAM sink (integration/do_voting_gpu.c), when linked */
int svg_sam_finish(void) __attribute__((weak));

int __wrap_write_indel_final_results(global_context_t *gc)
{
	if (svg_sam_finish && svg_sam_finish()) gc->output_sam_is_full = 1;
	double t0 = miltime();
	int rc = __real_write_indel_final_results(gc);
	if (getenv("SVG_REF_TIMING"))
		fprintf(stderr, "SVG_REF_PHASES load_index=%.6f voting=%.6f before_realign=%.6f realign=%.6f "
		        "write_vcf=%.6f wall=%.6f reads=%lld\n", gc->timecost_load_index, gc->timecost_voting,
		        gc->timecost_before_realign, gc->timecost_for_realign, miltime() - t0,
		        miltime() - gc->start_time, (long long)gc->all_processed_reads);
	return rc;
}

int __wrap_anti_supporting_read_scan(global_context_t *gc)
{
	/* SVG_REF_TIMING=1: the reference's own voting-phase clock (read_chunk_circles,
	 * core.c:3592-3595, cumulative over chunks; the print of core.c:480-485 is commented out
	 * in the reference) -- the CPU baseline calibration of tools/cpu_calibration.py */
	if (getenv("SVG_REF_TIMING"))
		fprintf(stderr, "SVG_REF_TIMECOST_VOTING %.6f %lld\n", gc->timecost_voting,
		        (long long)gc->processed_reads_in_chunk);
	const char *fn = getenv("SVG_REF_DUMP");
	if (fn && fn[0]) {
		FILE *fp = fopen(fn, "ab");
		if (fp) {
			long long n = gc->processed_reads_in_chunk, r;
			int ends = 1 + gc->input_reads.is_paired_end_reads;
			int mb = gc->config.multi_best_reads;
			for (r = 0; r < n; r++) {
				int e, b;
				for (e = 0; e < ends; e++)
					for (b = 0; b < mb; b++) {
						mapping_result_t m = *_global_retrieve_alignment_ptr(gc, r, e, b);
						m.result_flags &= ~CORE_IS_GAPPED_READ;
						fwrite(&m, sizeof(mapping_result_t), 1, fp);
					}
				if (gc->config.do_breakpoint_detection)
					for (e = 0; e < ends; e++)
						for (b = 0; b < mb; b++) {
							subjunc_result_t *j = _global_retrieve_subjunc_ptr(gc, r, e, b);
							fwrite(j, sizeof(subjunc_result_t), 1, fp);
						}
				if (gc->config.do_big_margin_filtering_for_junctions)
					for (e = 0; e < ends; e++) {
						unsigned short *bm = _global_retrieve_big_margin_ptr(gc, r, e);
						fwrite(bm, sizeof(unsigned short), gc->config.big_margin_record_size, fp);
					}
			}
			fclose(fp);
		}
	}
	int rc = __real_anti_supporting_read_scan(gc);
	/* the event table after the anti-supporting read scan (supporting counts unchanged by it) */
	const char *ef = getenv("SVG_REF_EVENTS");
	if (ef && ef[0]) dump_events(gc, ef);
	return rc;
}

/*
 * SVG_REF_READS_PER_CHUNK=N (tests only; the stock dump binary and the drop-ins alike): the
 * aligner's chunk size -- reads_per_chunk, 20M / multi_best (/ 2 for pairs) after
 * load_global_context (core.c:4091-4094) -- set to N in the first init_bigtable_results
 * (core.c:3837), before the bigtable is sized from it (core-bigtable.c:84-90).  A small test input
 * then runs as several read chunks, so the event table, the expected-TLEN estimate and the output
 * stream cross chunk boundaries (clean_context_after_chunk, core.c:3463-3478) as they do in a
 * run of more than 6.7M reads.
 */
int __real_init_bigtable_results(global_context_t *gc, int is_rewinding);
int __wrap_init_bigtable_results(global_context_t *gc, int is_rewinding)
{
	const char *e = getenv("SVG_REF_READS_PER_CHUNK");
	if (!is_rewinding && e && atol(e) > 0) gc->config.reads_per_chunk = atol(e);
	return __real_init_bigtable_results(gc, is_rewinding);
}
