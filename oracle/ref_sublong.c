/* TEST INFRASTRUCTURE ONLY -- never linked into the product.
 *
 * ref_sublong: the reference's own sublong voting step run over a FASTQ file and dumped.
 * Linked against the reference's longread-one objects compiled in place from
 * $(REF)/src/longread-one (oracle/Makefile; longread-mapping.c is compiled with -Dmain=... so
 * this file provides main).  For every read it runs exactly what LRMchunk_read_iteration does
 * before the dynamic-programming stage (longread-mapping.c:1343-1348, 1314-1317):
 *
 *   LRMdo_one_voting_read          (longread-mapping.c:552-560: both strands, LRMgehash_go_QQ
 *                                   per subread, LRMsorted-hashtable.c:443-518)
 *   LRMcopy_longvotes_to_itr       (longread-mapping.c:668-682: the table, row-major)
 *   LRMmerge_sort(... location ...) (longread-mapping.c:1317, LRMhelper.c:26-43)
 *
 * Output (binary, little-endian), per read:
 *   u32 n
 *   n x { u32 pos, u32 coverage_start, u32 coverage_end, u16 votes, u8 negative, u8 0, u32 bb<<16|ii }
 *       in LRMcopy_longvotes_to_itr's order
 *   n x u32: for sorted position k, the index (in the list above) of the entry sorted there
 *
 * usage: ref-sublong <index prefix> <reads.fastq> <out.bin>
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include "LRMconfig.h"
#include "LRMhelper.h"
#include "LRMsorted-hashtable.h"
#include "LRMfile-io.h"

void LRMdo_one_voting_read(LRMcontext_t *context, LRMthread_context_t *thread_context,
                           LRMread_iteration_context_t *iteration_context);
void LRMcopy_longvotes_to_itr(LRMcontext_t *context, LRMthread_context_t *thread_context,
                              LRMread_iteration_context_t *iteration_context);
int LRM_longvote_location_compare(void *arr, int l, int r);
void LRM_longvote_location_exchange(void *arr, int l, int r);
void LRM_longvote_location_merge(void *arr, int start, int items, int items2);

int main(int argc, char **argv)
{
	if (argc < 4) {
		fprintf(stderr, "usage: %s <index prefix> <reads.fastq> <out.bin>\n", argv[0]);
		return 2;
	}
	LRMcontext_t *ctx = calloc(1, sizeof(LRMcontext_t));
	LRMread_iteration_context_t *it = calloc(1, sizeof(LRMread_iteration_context_t));
	if (!ctx || !it) { fprintf(stderr, "out of memory\n"); return 1; }
	/* LRMset_default_values_context (longread-mapping.c:300): max_read_indel_length = 0 */
	ctx->max_read_indel_length = 0;
	char fn[LRMMAX_FILENAME_LENGTH + 20];
	snprintf(fn, sizeof fn, "%s.00.b.tab", argv[1]);
	if (LRMgehash_load(&ctx->current_index, fn)) { fprintf(stderr, "cannot load %s\n", fn); return 1; }
	LRMgene_input_t in;
	if (LRMgeinput_open(argv[2], &in)) { fprintf(stderr, "cannot open %s\n", argv[2]); return 1; }
	FILE *out = fopen(argv[3], "wb");
	if (!out) { fprintf(stderr, "cannot write %s\n", argv[3]); return 1; }
	static uint32_t map_key[LRMMAX_LOCATIONS_PER_READ_HARDLIMIT];
	long reads = 0;
	for (;;) {
		int rl = LRMgeinput_next_read(&in, it->read_name, it->read_text, it->qual_text);
		if (rl <= 0) break;   /* LRMfetch_next_read ends the input at the first empty read too */
		it->read_length = (unsigned)rl;
		LRMdo_one_voting_read(ctx, NULL, it);
		LRMcopy_longvotes_to_itr(ctx, NULL, it);
		const uint32_t n = it->sorting_total_votes;
		LRMgene_vote_t *v = &it->vote_table;
		fwrite(&n, 4, 1, out);
		for (uint32_t k = 0; k < n; k++) {
			const uint32_t s = it->sorting_subread_nos[k], bb = s >> 16, ii = s & 0xffff;
			uint8_t rec[20];
			const uint32_t pos = v->pos[bb][ii], cs = v->coverage_start[bb][ii], ce = v->coverage_end[bb][ii];
			const uint16_t votes = v->votes[bb][ii];
			memcpy(rec, &pos, 4);
			memcpy(rec + 4, &cs, 4);
			memcpy(rec + 8, &ce, 4);
			memcpy(rec + 12, &votes, 2);
			rec[14] = (uint8_t)it->sorting_is_negative_strand[k];
			rec[15] = 0;
			memcpy(rec + 16, &s, 4);
			fwrite(rec, 20, 1, out);
			map_key[k] = s;
		}
		/* the entries' keys bb<<16|ii are unique: remember each one's unsorted index */
		uint32_t *keys = malloc(sizeof(uint32_t) * (n ? n : 1));
		memcpy(keys, map_key, sizeof(uint32_t) * n);
		LRMmerge_sort(it, (int)n, LRM_longvote_location_compare, LRM_longvote_location_exchange,
		              LRM_longvote_location_merge);
		for (uint32_t k = 0; k < n; k++) {
			const uint32_t s = it->sorting_subread_nos[k];
			/* the flattened order is row-major (bb, ii): binary search it */
			uint32_t lo = 0, hi = n;
			while (lo < hi) { uint32_t m = (lo + hi) / 2; if (keys[m] < s) lo = m + 1; else hi = m; }
			fwrite(&lo, 4, 1, out);
		}
		free(keys);
		reads++;
	}
	fclose(out);
	LRMgeinput_close(&in);
	fprintf(stderr, "ref-sublong: %ld reads\n", reads);
	return 0;
}
