/* TEST INFRASTRUCTURE ONLY: the reference's own prefill_votes (cellCounts' hit-list lookup,
 * cell-counts.c:432-491), compiled from the reference source where it lies (this file
 * #includes it; nothing is copied), driven over a subread-buildindex index block.
 *
 *   ref-prefill <index prefix> <block> <keys.u32 file> <out file>
 *
 * For every little-endian u32 key of <keys file> it writes two u32 to <out file>: the
 * bucket-local index of the run's first item (start_location_in_index - bucket->item_values,
 * 0 when absent) and votes (the run length, 0 when absent) -- the outputs svg_probe_keys
 * must reproduce. */
#define main cellcounts_unused_main
#include REF_CELL_COUNTS
#undef main

int main(int argc, char **argv)
{
	if (argc != 5) { fprintf(stderr, "usage: %s prefix block keys.u32 out.u32\n", argv[0]); return 2; }
	char tab[1030];
	snprintf(tab, sizeof tab, "%s.%02d.b.tab", argv[1], atoi(argv[2]));
	gehash_t table;
	if (gehash_load(&table, tab)) { fprintf(stderr, "cannot load %s\n", tab); return 1; }
	FILE *fk = fopen(argv[3], "rb"), *fo = fopen(argv[4], "wb");
	if (!fk || !fo) { fprintf(stderr, "cannot open key / output file\n"); return 1; }
	temp_votes_per_read_t *pnts = calloc(1, sizeof *pnts);
	unsigned int key;
	while (fread(&key, 4, 1, fk) == 1) {
		pnts->votes[0] = 0;
		pnts->start_location_in_index[0] = NULL;
		prefill_votes(&table, pnts, 1, key, 0, 0, 0);
		struct gehash_bucket *b = table.buckets + key % table.buckets_number;
		unsigned int o[2];
		o[1] = (unsigned int)pnts->votes[0];
		o[0] = o[1] ? (unsigned int)(pnts->start_location_in_index[0] - b->item_values) : 0u;
		fwrite(o, 4, 2, fo);
	}
	fclose(fk);
	fclose(fo);
	free(pnts);
	gehash_destory(&table);
	return 0;
}
