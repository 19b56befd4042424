/*
 * svg_build.c -- format-exact builder of the Subread base-space index
 * (<prefix>.NN.b.tab / .NN.b.array / .reads / .files / .log), one block or several.
 *
 * Replaces subread-buildindex (index-builder.c:1014-1306) for the one-block
 * case: the bytes of .tab/.array/.reads equal the reference's (md5 known
 * answers in tests/golden/index_md5.json).  The reference builds the table by
 * per-bucket insertion + selection sort at dump time; here the same total order
 * is produced with two LSD radix sorts:
 *   1. FASTA normalisation     check_and_convert_FastA   index-builder.c:789-992
 *      (a/c/g/t any case -> upper, everything else -> 'A'; contigs <=16 bp dropped)
 *   2. coordinates             build_gene_index          index-builder.c:113-420
 *      (first contig at PAD=1210, next at +L-16+2*PAD; .reads = O+L-16+PAD)
 *   3. sampled 16-mers every `gap` bases, key = genekey2int (input-files.c:1232)
 *   4. repeat exclusion        scan_gene_index           index-builder.c:472-684
 *      (keys occurring > threshold times over the sampled windows are dropped)
 *   5. bucket count            calculate_buckets_by_size sorted-hashtable.c:42-75
 *   6. .tab layout + in-bucket order  gehash_dump / is_1_greater_than_2
 *                                      sorted-hashtable.c:1689-1908
 *   7. .array 2-bit LSB-first  gvindex_set / gvindex_dump gene-value-index.c:135-187
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <ctype.h>
#include <unistd.h>
#include <zlib.h>
#include "subread_vote.h"
#include "svg_internal.h"

#define PAD 1210
#define NAME_MAX_LEN 200

typedef svg_contig contig_t;
typedef svg_genome genome_t;

static void g_push(genome_t *g, const char *s, size_t n)
{
	if (g->nbases + n > g->cap) {
		g->cap = (g->nbases + n) * 2 + (1 << 20);
		g->bases = realloc(g->bases, g->cap);
	}
	memcpy(g->bases + g->nbases, s, n);
	g->nbases += n;
}

/* check_and_convert_FastA semantics (index-builder.c:789-992) */
int svg_genome_read_fasta(const char *path, genome_t *g)
{
	gzFile fp = gzopen(path, "rb");
	char *line = malloc(1 << 16);
	int have = 0;
	if (!fp) { free(line); svg_set_error("cannot open FASTA '%s'", path); return SVG_E_IO; }
	while (gzgets(fp, line, 1 << 16)) {
		size_t L = strlen(line);
		while (L && (line[L - 1] == '\n' || line[L - 1] == '\r')) line[--L] = 0;
		if (!L) continue;
		if (line[0] == '>') {
			contig_t *c;
			uint32_t i;
			if (have && g->ctg[g->nctg - 1].len <= 16) {  /* short contig: drop entirely */
				g->nbases = g->ctg[g->nctg - 1].start;
				g->nctg--;
			}
			if (g->nctg == g->ctg_cap) {
				g->ctg_cap = g->ctg_cap ? g->ctg_cap * 2 : 64;
				g->ctg = realloc(g->ctg, sizeof(contig_t) * g->ctg_cap);
			}
			c = &g->ctg[g->nctg++];
			memset(c, 0, sizeof *c);
			/* .reads name: up to ' ', '\t' or end, at most NAME_MAX_LEN-1 chars
			 * (build_gene_index, index-builder.c:266-270, '|' kept) */
			for (i = 0; line[i + 1] && line[i + 1] != ' ' && line[i + 1] != '\t' && i < NAME_MAX_LEN - 1; i++)
				c->name[i] = line[i + 1];
			c->name[i] = 0;
			/* duplicate names are an error in the reference */
			{
				uint32_t k;
				char key[NAME_MAX_LEN]; size_t kl = 0;
				for (kl = 0; line[kl + 1] && line[kl + 1] != ' ' && line[kl + 1] != '|' && line[kl + 1] != '\t' && kl < NAME_MAX_LEN - 1; kl++) key[kl] = line[kl + 1];
				key[kl] = 0;
				for (k = 0; k + 1 < g->nctg; k++) {
					char k2[NAME_MAX_LEN]; size_t j;
					for (j = 0; g->ctg[k].name[j] && g->ctg[k].name[j] != '|' && j < NAME_MAX_LEN - 1; j++) k2[j] = g->ctg[k].name[j];
					k2[j] = 0;
					if (!strcmp(k2, key)) { gzclose(fp); free(line); svg_set_error("repeated chromosome name '%s'", key); return SVG_E_FORMAT; }
				}
			}
			c->start = g->nbases;
			have = 1;
		} else if (have) {
			size_t i;
			for (i = 0; i < L; i++) {
				int ch = line[i], lo = tolower(ch);
				if (lo == 'a' || lo == 'c' || lo == 'g' || lo == 't') line[i] = (char)toupper(ch);
				else line[i] = 'A';
			}
			g_push(g, line, L);
			g->ctg[g->nctg - 1].len += (uint32_t)L;
		}
	}
	if (have && g->ctg[g->nctg - 1].len <= 16) { g->nbases = g->ctg[g->nctg - 1].start; g->nctg--; }
	gzclose(fp);
	free(line);
	if (!g->nctg) { svg_set_error("no contig of >16 bases in '%s'", path); return SVG_E_FORMAT; }
	return 0;
}

/* calculate_buckets_by_size, sorted-hashtable.c:42-75 (VER2) */
uint32_t svg_bucket_count(uint64_t expected_items, int gap)
{
	int64_t nb = (int64_t)(expected_items / 31);
	if (gap >= 3) nb /= 3;
	if (nb <= 0x3ffff) nb = 0x3ffff + 4;
	for (;; nb++) {
		int j, ok = 1;
		for (j = 2; j <= 13; j++) if (nb % j == 0) ok = 0;
		if (ok) break;
	}
	return (uint32_t)nb;
}

static inline uint32_t b2i(char c) { return c < 'G' ? (c == 'A' ? 0 : 2) : (c == 'G' ? 1 : 3); }

/* LSD radix sort of 64-bit keys, 16-bit digits, skipping constant digits */
static void radix64(uint64_t *a, uint64_t *tmp, uint64_t n)
{
	int pass;
	uint64_t *cnt = malloc(sizeof(uint64_t) * 65536);
	for (pass = 0; pass < 4; pass++) {
		int sh = pass * 16;
		uint64_t i, s = 0;
		memset(cnt, 0, sizeof(uint64_t) * 65536);
		for (i = 0; i < n; i++) cnt[(a[i] >> sh) & 0xffff]++;
		for (i = 0; i < 65536; i++) if (cnt[i] == n) break;
		if (i < 65536) continue;   /* digit constant -> already ordered */
		for (i = 0; i < 65536; i++) { uint64_t c = cnt[i]; cnt[i] = s; s += c; }
		for (i = 0; i < n; i++) tmp[cnt[(a[i] >> sh) & 0xffff]++] = a[i];
		memcpy(a, tmp, n * sizeof(uint64_t));
	}
	free(cnt);
}

static int write_all(FILE *fp, const void *p, size_t n) { return fwrite(p, 1, n, fp) == n ? 0 : -1; }

void svg_genome_free(genome_t *g)
{
	free(g->bases); free(g->ctg);
	memset(g, 0, sizeof *g);
}

/* in-memory contigs -> normalised genome (same rules as the FASTA path) */
int svg_genome_from_mem(const char *const *names, const char *const *seqs, const uint64_t *lens, uint32_t n, genome_t *g)
{
	uint32_t c;
	memset(g, 0, sizeof *g);
	for (c = 0; c < n; c++) {
		uint64_t i;
		contig_t *ct;
		if (lens[c] <= 16) continue;
		if (lens[c] > 0xffffffffull) { svg_set_error("contig longer than 2^32"); return SVG_E_UNSUPPORTED; }
		if (g->nctg == g->ctg_cap) {
			g->ctg_cap = g->ctg_cap ? g->ctg_cap * 2 : 64;
			g->ctg = realloc(g->ctg, sizeof(contig_t) * g->ctg_cap);
		}
		ct = &g->ctg[g->nctg++];
		memset(ct, 0, sizeof *ct);
		snprintf(ct->name, NAME_MAX_LEN, "%s", names[c]);
		ct->start = g->nbases;
		ct->len = (uint32_t)lens[c];
		if (g->nbases + lens[c] > g->cap) {
			g->cap = g->nbases + lens[c] + (1 << 20);
			g->bases = realloc(g->bases, g->cap);
		}
		for (i = 0; i < lens[c]; i++) {
			int ch = seqs[c][i], lo = tolower(ch);
			g->bases[g->nbases + i] = (lo == 'a' || lo == 'c' || lo == 'g' || lo == 't') ? (char)toupper(ch) : 'A';
		}
		g->nbases += lens[c];
	}
	if (!g->nctg) { svg_set_error("no contig of >16 bases"); return SVG_E_FORMAT; }
	return 0;
}

void svg_genome_layout(const genome_t *g, int gap, uint64_t *O, uint64_t *nwin)
{
	uint64_t off = PAD;
	uint32_t c;
	*nwin = 0;
	for (c = 0; c < g->nctg; c++) {
		O[c] = off;
		*nwin += (g->ctg[c].len - 16) / gap + 1;
		off += (uint64_t)g->ctg[c].len - 16 + 2 * PAD;
	}
}

uint64_t svg_items_budget(int gap, int memory_mb, int force_one_block)
{
	if (force_one_block) memory_mb = gap == 1 ? 22000 : 11500;
	else if (memory_mb > 12000 && gap > 2) memory_mb = 12000;
	return (uint32_t)(memory_mb * 1024.0 / 8.) * 1024;
}

static int write_tab_block(const char *prefix, int block, uint32_t nb, uint64_t items, int gap, const uint32_t *bstart,
                           const int16_t *keys, const uint32_t *vals)
{
	char fn[4096];
	FILE *fp;
	char *buf;
	size_t bufsz = 1 << 24, bl = 0;
	uint32_t c;
	int rc = 0;
	snprintf(fn, sizeof fn, "%s.%02d.b.tab", prefix, block);
	fp = fopen(fn, "wb");
	if (!fp) { svg_set_error("cannot write '%s'", fn); return SVG_E_IO; }
	buf = malloc(bufsz);
	{
		int16_t opt[7] = {0x0102, 2, PAD, 0x0101, 2, (int16_t)gap, 0};
		int64_t nit = (int64_t)items; int32_t nbs = (int32_t)nb;
		memcpy(buf + bl, "2subindx", 8); bl += 8;
		memcpy(buf + bl, opt, sizeof opt); bl += sizeof opt;
		memcpy(buf + bl, &nit, 8); bl += 8;
		memcpy(buf + bl, &nbs, 4); bl += 4;
	}
	for (c = 0; c < nb && !rc; c++) {
		int32_t n = (int32_t)(bstart[c + 1] - bstart[c]);
		size_t need = 8 + 6 * (size_t)n;
		if (bl + need > bufsz) {
			if (write_all(fp, buf, bl)) rc = SVG_E_IO;
			bl = 0;
			if (need > bufsz) { bufsz = need * 2; buf = realloc(buf, bufsz); }
		}
		memcpy(buf + bl, &n, 4); memcpy(buf + bl + 4, &n, 4); bl += 8;
		memcpy(buf + bl, keys + bstart[c], 2 * (size_t)n); bl += 2 * (size_t)n;
		memcpy(buf + bl, vals + bstart[c], 4 * (size_t)n); bl += 4 * (size_t)n;
	}
	buf[bl++] = 0;
	if (!rc && write_all(fp, buf, bl)) rc = SVG_E_IO;
	if (fclose(fp)) rc = SVG_E_IO;
	free(buf);
	if (rc) svg_set_error("write error on '%s'", fn);
	return rc;
}

int svg_write_tab(const char *prefix, uint32_t nb, uint64_t items, int gap, const uint32_t *bstart,
                  const int16_t *keys, const uint32_t *vals)
{
	return write_tab_block(prefix, 0, nb, items, gap, bstart, keys, vals);
}

/* blocks a previous build into the same prefix left behind (build_gene_index, index-builder.c:181-187) */
static void unlink_blocks_from(const char *prefix, int first)
{
	char fn[4096];
	int i;
	for (i = first; i < 100; i++) {
		snprintf(fn, sizeof fn, "%s.%02d.b.tab", prefix, i);
		unlink(fn);
		snprintf(fn, sizeof fn, "%s.%02d.b.array", prefix, i);
		unlink(fn);
	}
}

uint8_t *svg_pack_array(const genome_t *g, const uint64_t *O, uint32_t *length_out, uint32_t *vbytes_out)
{
	uint32_t last = g->nctg - 1, c;
	uint32_t length = (uint32_t)(O[last] + g->ctg[last].len - 16 + 16 + PAD);
	size_t nbytes = (length >> 2) + 1;
	uint8_t *arr = calloc(nbytes + 64, 1);
	if (!arr) return NULL;
	for (c = 0; c < g->nctg; c++) {
		const char *b = g->bases + g->ctg[c].start;
		uint32_t k;
		for (k = 0; k < g->ctg[c].len; k++) {
			uint64_t p = O[c] + k;
			arr[p >> 2] |= (uint8_t)(b2i(b[k]) << (2 * (p & 3)));
		}
	}
	*length_out = length;
	*vbytes_out = (uint32_t)nbytes;
	return arr;
}

static int write_array_block(const char *prefix, int block, uint32_t start, uint32_t length, const uint8_t *arr, size_t vb)
{
	char fn[4096];
	FILE *fp;
	int rc = 0;
	snprintf(fn, sizeof fn, "%s.%02d.b.array", prefix, block);
	fp = fopen(fn, "wb");
	if (!fp) { svg_set_error("cannot write '%s'", fn); return SVG_E_IO; }
	if (write_all(fp, &start, 4) || write_all(fp, &length, 4) || write_all(fp, arr, vb)) rc = SVG_E_IO;
	if (fclose(fp)) rc = SVG_E_IO;
	if (rc) svg_set_error("write error on '%s'", fn);
	return rc;
}

/* .reads / .files / .log (the genome-wide files of any build) */
static int write_reads_files(const char *prefix, const genome_t *g, const uint64_t *O, int gap, uint64_t nwin,
                             uint64_t items, uint32_t nb, int nblocks, const char *source)
{
	char fn[4096];
	FILE *fp;
	uint32_t c;
	snprintf(fn, sizeof fn, "%s.reads", prefix);
	fp = fopen(fn, "wb");
	if (!fp) { svg_set_error("cannot write '%s'", fn); return SVG_E_IO; }
	for (c = 0; c < g->nctg; c++) fprintf(fp, "%u\t%s\n", (uint32_t)(O[c] + g->ctg[c].len - 16 + PAD), g->ctg[c].name);
	fclose(fp);
	snprintf(fn, sizeof fn, "%s.files", prefix);
	fp = fopen(fn, "wb");
	if (fp) { for (c = 0; c < g->nctg; c++) fprintf(fp, "%s\t%s\t0\n", g->ctg[c].name, source); fclose(fp); }
	snprintf(fn, sizeof fn, "%s.log", prefix);
	fp = fopen(fn, "wb");
	if (fp) {
		fprintf(fp, "svg index: %u contigs, %llu windows, %llu items, %u buckets, gap %d, %d block%s\n", g->nctg,
		        (unsigned long long)nwin, (unsigned long long)items, nb, gap, nblocks, nblocks > 1 ? "s" : "");
		fclose(fp);
	}
	return 0;
}

int svg_write_array_reads(const char *prefix, const genome_t *g, const uint64_t *O, int gap, uint64_t nwin,
                          uint64_t items, uint32_t nb, const char *source)
{
	uint32_t length, vb;
	int rc;
	uint8_t *arr = svg_pack_array(g, O, &length, &vb);
	if (!arr) { svg_set_error("out of memory packing .array"); return SVG_E_NOMEM; }
	rc = write_array_block(prefix, 0, 0, length, arr, vb);
	free(arr);
	if (rc) return rc;
	unlink_blocks_from(prefix, 1);
	return write_reads_files(prefix, g, O, gap, nwin, items, nb, 1, source);
}

/* sorted (key << 32 | pa) items -> bucket layout -> <prefix>.NN.b.tab (gehash_dump,
 * sorted-hashtable.c:1689-1908): a stable counting sort by bucket keeps the key/pa order */
static int tab_from_sorted(const char *prefix, int block, uint32_t nb, const uint64_t *items, uint64_t n, int gap)
{
	uint64_t i;
	uint32_t c;
	int rc;
	uint32_t *bstart = calloc((size_t)nb + 1, sizeof(uint32_t));
	int16_t *keys = malloc(2 * n + 2);
	uint32_t *vals = malloc(4 * n + 4);
	uint32_t *cur = malloc(sizeof(uint32_t) * nb);
	if (!bstart || !keys || !vals || !cur) {
		free(bstart); free(keys); free(vals); free(cur);
		svg_set_error("out of memory laying out the table");
		return SVG_E_NOMEM;
	}
	for (i = 0; i < n; i++) bstart[(uint32_t)(items[i] >> 32) % nb + 1]++;
	for (c = 0; c < nb; c++) bstart[c + 1] += bstart[c];
	memcpy(cur, bstart, sizeof(uint32_t) * nb);
	for (i = 0; i < n; i++) {
		uint32_t key = (uint32_t)(items[i] >> 32), pa = (uint32_t)items[i];
		uint32_t b = key % nb, d = cur[b]++;
		keys[d] = (int16_t)(key / nb);
		vals[d] = ((key % 791) % 2 == 0) ? pa : ~pa;
	}
	free(cur);
	rc = write_tab_block(prefix, block, nb, n, gap, bstart, keys, vals);
	free(bstart); free(keys); free(vals);
	return rc;
}

static inline uint32_t window_key(const char *b)
{
	uint32_t key = 0;
	int k;
	for (k = 0; k < 16; k++) key |= b2i(b[k]) << (30 - 2 * k);
	return key;
}

/* is_1_greater_than_2: equal keys ascending by pos if key%791 even, else descending */
static inline uint64_t window_item(uint32_t key, uint32_t pos)
{
	return ((uint64_t)key << 32) | (((key % 791) % 2 == 0) ? pos : ~pos);
}

static int is_repeat(const uint32_t *rep, uint64_t nrep, uint32_t key)
{
	uint64_t lo = 0, hi = nrep;
	while (lo < hi) {
		uint64_t m = (lo + hi) / 2;
		if (rep[m] < key) lo = m + 1; else hi = m;
	}
	return lo < nrep && rep[lo] == key;
}

/*
 * Multi-block build (build_gene_index, index-builder.c:257-357): windows are inserted in genome
 * order; once a block holds `budget` items it is closed at the next window whose read_len (16 +
 * distance from the contig start) is < 32 -- the block then restarts that contig from its first
 * base -- or > MIN_READ_SPLICING (2,000,000) -- the next block then starts 1,999,974 bases back,
 * so both hold the overlap.  Every block has its own .tab (same bucket count) and its own .array
 * (start_point = the block's first window; the bases its windows and contig-end writes covered,
 * gvindex_set / gvindex_dump, gene-value-index.c:135-187).
 */
typedef struct { uint32_t c; uint64_t a, b; int ends; } seg_t;
typedef struct { uint64_t start, last_set, items; uint32_t s0, ns; } blk_t;

#define MIN_READ_SPLICING 2000000u
#define SPLICE_BACK (MIN_READ_SPLICING - 10 - (MIN_READ_SPLICING - 10) % 3 + 1 - 16)

static int build_blocks(const char *prefix, const genome_t *g, const uint64_t *O, int gap, uint32_t nb, uint64_t budget,
                        const uint32_t *rep, uint64_t nrep, int *nblocks_out)
{
	seg_t *seg = NULL;
	blk_t *blk = NULL;
	uint32_t nseg = 0, segcap = 0, nblk = 0, blkcap = 0, c, k;
	int rc = 0;
#define PUSH_SEG(C, A, B, E) do { \
		if (nseg == segcap) { segcap = segcap ? 2 * segcap : 64; seg = realloc(seg, sizeof(seg_t) * segcap); } \
		seg[nseg].c = (C); seg[nseg].a = (A); seg[nseg].b = (B); seg[nseg].ends = (E); nseg++; blk[nblk - 1].ns++; } while (0)
#define NEW_BLOCK(S) do { \
		if (nblk == blkcap) { blkcap = blkcap ? 2 * blkcap : 16; blk = realloc(blk, sizeof(blk_t) * blkcap); } \
		blk[nblk].start = (S); blk[nblk].items = 0; blk[nblk].s0 = nseg; blk[nblk].ns = 0; blk[nblk].last_set = 0; nblk++; } while (0)
	NEW_BLOCK(0);
	for (c = 0; c < g->nctg; c++) {
		const char *base = g->bases + g->ctg[c].start;
		const uint64_t last = O[c] + (uint64_t)((g->ctg[c].len - 16) / gap) * gap;
		uint64_t p = O[c], a = O[c];
		while (p <= last) {
			const uint64_t rl = 16 + p - O[c];
			if (!is_repeat(rep, nrep, window_key(base + (p - O[c])))) blk[nblk - 1].items++;
			if (blk[nblk - 1].items >= budget && (rl > MIN_READ_SPLICING || rl < 32)) {
				PUSH_SEG(c, a, p, 0);
				blk[nblk - 1].last_set = p;
				if (nblk == 100) {   /* a budget far below MIN_READ_SPLICING items can cycle forever */
					rc = SVG_E_UNSUPPORTED;
					svg_set_error("more than 100 index blocks: raise memory_mb");
					goto out;
				}
				p = rl < 32 ? O[c] : p - SPLICE_BACK;
				NEW_BLOCK(p);
				a = p;
				continue;
			}
			p += gap;
		}
		PUSH_SEG(c, a, last, 1);
		blk[nblk - 1].last_set = O[c] + g->ctg[c].len - 16;
	}
#undef PUSH_SEG
#undef NEW_BLOCK
	for (k = 0; k < nblk && !rc; k++) {
		const blk_t *B = &blk[k];
		uint64_t *items = malloc(sizeof(uint64_t) * (B->items + 1)), *tmp = malloc(sizeof(uint64_t) * (B->items + 1)), n = 0;
		const uint64_t sbo = B->start - B->start % 4;
		const uint32_t length = (uint32_t)(B->last_set + 16 - B->start + PAD);
		const size_t vb = (size_t)((length + B->start - sbo) >> 2) + 1;
		uint8_t *arr = calloc(vb + 8, 1);
		uint32_t s;
		if (!items || !tmp || !arr) { free(items); free(tmp); free(arr); rc = SVG_E_NOMEM; svg_set_error("out of memory (block %u)", k); break; }
		for (s = B->s0; s < B->s0 + B->ns; s++) {
			const seg_t *S = &seg[s];
			const char *base = g->bases + g->ctg[S->c].start;
			const uint64_t set_end = S->ends ? O[S->c] + g->ctg[S->c].len : S->b + 16;
			uint64_t p;
			for (p = S->a; p <= S->b; p += gap) {
				uint32_t key = window_key(base + (p - O[S->c]));
				if (!is_repeat(rep, nrep, key)) items[n++] = window_item(key, (uint32_t)p);
			}
			for (p = S->a; p < set_end; p++) arr[(p - sbo) >> 2] |= (uint8_t)(b2i(base[p - O[S->c]]) << (2 * (p & 3)));
		}
		radix64(items, tmp, n);
		free(tmp);
		rc = tab_from_sorted(prefix, (int)k, nb, items, n, gap);
		free(items);
		if (!rc) rc = write_array_block(prefix, (int)k, (uint32_t)B->start, length, arr, vb);
		free(arr);
	}
	if (!rc) unlink_blocks_from(prefix, (int)nblk);
	*nblocks_out = (int)nblk;
out:
	free(seg); free(blk);
	return rc;
}

int svg_build_index(const char *fasta, const char *prefix, int gap, int memory_mb, int force_one_block, int repeat_threshold)
{
	genome_t g;
	uint64_t *O = NULL, nwin = 0, i, nkeep = 0;
	uint64_t *items = NULL, *tmp = NULL, nrep = 0, repcap = 0;
	uint32_t *rep = NULL;
	uint32_t c, nb;
	uint64_t budget;
	int rc = 0;
	memset(&g, 0, sizeof g);
	if (!fasta || !prefix || (gap != 1 && gap != 3)) { svg_set_error("svg_build_index: bad argument"); return SVG_E_ARG; }
	if (repeat_threshold < 1) repeat_threshold = 100;
	rc = svg_genome_read_fasta(fasta, &g);
	if (rc) goto out;

	/* 2. coordinates */
	O = malloc(sizeof(uint64_t) * g.nctg);
	svg_genome_layout(&g, gap, O, &nwin);
	if (O[g.nctg - 1] + g.ctg[g.nctg - 1].len + PAD >= 0xffffffffull) { rc = SVG_E_UNSUPPORTED; svg_set_error("genome too long for 32-bit coordinates"); goto out; }

	/* 5. bucket count */
	budget = svg_items_budget(gap, memory_mb, force_one_block);
	nb = svg_bucket_count(budget, gap);

	/* 3+4. windows, sorted by (key, in-run order) */
	items = malloc(sizeof(uint64_t) * (nwin + 1));
	tmp = malloc(sizeof(uint64_t) * (nwin + 1));
	if (!items || !tmp) { rc = SVG_E_NOMEM; svg_set_error("out of memory (%llu windows)", (unsigned long long)nwin); goto out; }
	{
		uint64_t w = 0;
		for (c = 0; c < g.nctg; c++) {
			const char *b = g.bases + g.ctg[c].start;
			uint32_t t, nt = (g.ctg[c].len - 16) / gap + 1;
			for (t = 0; t < nt; t++) {
				uint32_t key = 0, pos = (uint32_t)(O[c] + (uint64_t)t * gap), pa; int k;
				for (k = 0; k < 16; k++) key |= b2i(b[(uint64_t)t * gap + k]) << (30 - 2 * k);
				/* is_1_greater_than_2: equal keys ascending by pos if key%791 even, else descending */
				pa = ((key % 791) % 2 == 0) ? pos : ~pos;
				items[w++] = ((uint64_t)key << 32) | pa;
			}
		}
	}
	radix64(items, tmp, nwin);
	/* drop keys occurring more than repeat_threshold times (the repeated keys are kept, in order,
	 * for a multi-block build) */
	for (i = 0; i < nwin;) {
		uint64_t j = i;
		uint32_t key = (uint32_t)(items[i] >> 32);
		while (j < nwin && (uint32_t)(items[j] >> 32) == key) j++;
		if (j - i <= (uint64_t)repeat_threshold) {
			uint64_t k;
			for (k = i; k < j; k++) items[nkeep++] = items[k];
		} else {
			if (nrep == repcap) { repcap = repcap ? 2 * repcap : 1024; rep = realloc(rep, sizeof(uint32_t) * repcap); }
			rep[nrep++] = key;
		}
		i = j;
	}
	if (!force_one_block && nkeep >= budget) {
		/* may still come out as one block: splits happen only near contig starts or deep in contigs */
		int nblocks = 0;
		free(items); items = NULL;
		free(tmp); tmp = NULL;
		rc = build_blocks(prefix, &g, O, gap, nb, budget, rep, nrep, &nblocks);
		if (!rc) rc = write_reads_files(prefix, &g, O, gap, nwin, nkeep, nb, nblocks, fasta);
		goto out;
	}
	if (nkeep > 0xffffffffull) { rc = SVG_E_UNSUPPORTED; svg_set_error("more than 2^32-1 items"); goto out; }

	/* 6. stable counting sort by bucket (within a bucket, key order == key_hi order) */
	free(tmp); tmp = NULL;
	rc = tab_from_sorted(prefix, 0, nb, items, nkeep, gap);
	free(items); items = NULL;
	if (rc) goto out;
	rc = svg_write_array_reads(prefix, &g, O, gap, nwin, nkeep, nb, fasta);
out:
	free(items); free(tmp); free(O); free(rep);
	svg_genome_free(&g);
	return rc;
}
