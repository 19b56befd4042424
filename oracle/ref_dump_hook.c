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

int __real_anti_supporting_read_scan(global_context_t *global_context);

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
	return __real_anti_supporting_read_scan(gc);
}
