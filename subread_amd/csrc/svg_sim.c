/*
 * svg_sim.c -- seeded synthetic genomes and reads for tests and benchmarks
 * (the counterpart of the reference's genRandomReads utility, gen_rand_reads.c).
 *
 * Every random draw is a pure function of (seed, read number, draw number), so
 * the output is identical for any thread count and any batch split.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <pthread.h>
#include "subread_vote.h"

static inline uint64_t mix64(uint64_t z)
{
	z += 0x9e3779b97f4a7c15ull;
	z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
	z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
	return z ^ (z >> 31);
}

typedef struct { uint64_t s; } rng_t;
static inline uint64_t rnext(rng_t *r) { r->s += 0x9e3779b97f4a7c15ull; return mix64(r->s); }
static inline double runif(rng_t *r) { return (rnext(r) >> 11) * (1.0 / 9007199254740992.0); }

static const char ACGT[4] = {'A', 'C', 'G', 'T'};

/* i.i.d. uniform ACGT genome of `length` bases (chunked by 1 Mbp for determinism) */
void svg_sim_genome(char *out, uint64_t length, uint64_t seed)
{
	uint64_t c;
	for (c = 0; c * 1048576ull < length; c++) {
		rng_t r = {mix64(seed * 0x100000001b3ull + c)};
		uint64_t i, e = (c + 1) * 1048576ull < length ? (c + 1) * 1048576ull : length;
		for (i = c * 1048576ull; i < e;) {
			uint64_t v = rnext(&r);
			int k;
			for (k = 0; k < 32 && i < e; k++, i++) out[i] = ACGT[(v >> (2 * k)) & 3];
		}
	}
}

/* copy `n` repeat-family elements (length elen, divergence div) over the genome */
void svg_sim_repeats(char *g, uint64_t length, uint64_t n_copies, uint32_t elen, uint32_t n_families, double div, uint64_t seed)
{
	uint64_t i;
	char *fam;
	uint32_t f;
	if (!n_families || elen == 0 || elen > length) return;
	fam = malloc((size_t)n_families * elen);
	for (f = 0; f < n_families; f++) {
		rng_t r = {mix64(seed ^ (0xabcdefull + f))};
		uint32_t k;
		for (k = 0; k < elen; k++) fam[(size_t)f * elen + k] = ACGT[rnext(&r) & 3];
	}
	for (i = 0; i < n_copies; i++) {
		rng_t r = {mix64(seed * 31 + i)};
		uint64_t at = rnext(&r) % (length - elen);
		const char *src = fam + (size_t)(rnext(&r) % n_families) * elen;
		uint32_t k;
		for (k = 0; k < elen; k++) {
			char b = src[k];
			if (runif(&r) < div) b = ACGT[rnext(&r) & 3];
			g[at + k] = b;
		}
	}
	free(fam);
}

static inline char compl(char c)
{
	switch (c) { case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A'; }
	return 'N';
}

typedef struct {
	const char *genome;
	const uint64_t *ctg_start;   /* start of contig c in `genome` */
	const uint64_t *ctg_cum;     /* cumulative usable start positions */
	uint32_t n_ctg;
	uint64_t n_reads, first;
	int len;
	double sub, indel, nrate;
	uint64_t seed;
	char *seq;
	uint32_t *t_ctg, *t_pos;
	uint8_t *t_strand;
	uint64_t r0, r1;
} sim_job;

static void *sim_worker(void *arg)
{
	sim_job *j = arg;
	uint64_t i;
	char buf[4096];
	for (i = j->r0; i < j->r1; i++) {
		uint64_t id = j->first + i;
		rng_t r = {mix64(j->seed ^ mix64(id))};
		uint64_t u = rnext(&r) % j->ctg_cum[j->n_ctg];
		uint32_t lo = 0, hi = j->n_ctg - 1;
		uint64_t pos;
		int L = j->len, k, o = 0, strand;
		char *dst = j->seq + i * (uint64_t)L;
		while (lo < hi) { uint32_t m = (lo + hi) / 2; if (j->ctg_cum[m + 1] <= u) lo = m + 1; else hi = m; }
		pos = u - j->ctg_cum[lo];
		{
			const char *src = j->genome + j->ctg_start[lo] + pos;
			int ilen = 0, at = -1, del = 0;
			if (runif(&r) < j->indel) {
				ilen = 1 + (int)(rnext(&r) % 5);
				del = (int)(rnext(&r) & 1);
				at = 10 + (int)(rnext(&r) % (uint64_t)(L - 20));
			}
			for (k = 0; o < L; k++) {
				if (k == at && !del) { int q; for (q = 0; q < ilen && o < L; q++) buf[o++] = ACGT[rnext(&r) & 3]; }
				if (k == at && del) k += ilen;
				if (o < L) buf[o++] = src[k];
			}
		}
		for (k = 0; k < L; k++) {
			if (runif(&r) < j->sub) { char b; do b = ACGT[rnext(&r) & 3]; while (b == buf[k]); buf[k] = b; }
			if (j->nrate > 0 && runif(&r) < j->nrate) buf[k] = 'N';
		}
		strand = (int)(rnext(&r) & 1);
		if (strand) for (k = 0; k < L; k++) dst[k] = compl(buf[L - 1 - k]);
		else memcpy(dst, buf, L);
		if (j->t_ctg) j->t_ctg[i] = lo;
		if (j->t_pos) j->t_pos[i] = (uint32_t)pos;
		if (j->t_strand) j->t_strand[i] = (uint8_t)strand;
	}
	return NULL;
}

/*
 * n_reads reads of length len, reads number first..first+n_reads-1 of the
 * stream defined by seed.  Reads start uniformly over the contig positions
 * that leave len+5 bases; 1 indel (1-5 bp) with probability indel_frac;
 * substitutions with probability sub per base; 'N' with probability nrate;
 * strand 50/50 (reverse-complemented).  Output: seq[n_reads*len] ASCII,
 * truth contig / 0-based position / strand (any may be NULL).
 */
int svg_sim_reads(const char *genome, const uint64_t *ctg_start, const uint32_t *ctg_len, uint32_t n_ctg,
                  uint64_t first, uint64_t n_reads, int len, double sub, double indel_frac, double nrate,
                  uint64_t seed, char *seq, uint32_t *t_ctg, uint32_t *t_pos, uint8_t *t_strand, int threads)
{
	uint64_t *cum;
	uint32_t c;
	int t;
	pthread_t th[256];
	sim_job jb[256];
	if (len < 32 || len > 4000 || !n_ctg) return SVG_E_ARG;
	cum = malloc(sizeof(uint64_t) * (n_ctg + 1));
	cum[0] = 0;
	for (c = 0; c < n_ctg; c++) cum[c + 1] = cum[c] + (ctg_len[c] > (uint32_t)len + 6 ? ctg_len[c] - len - 6 : 0);
	if (!cum[n_ctg]) { free(cum); return SVG_E_ARG; }
	if (threads < 1) threads = 1;
	if (threads > 256) threads = 256;
	for (t = 0; t < threads; t++) {
		jb[t].genome = genome; jb[t].ctg_start = ctg_start; jb[t].ctg_cum = cum; jb[t].n_ctg = n_ctg;
		jb[t].n_reads = n_reads; jb[t].first = first; jb[t].len = len; jb[t].sub = sub; jb[t].indel = indel_frac;
		jb[t].nrate = nrate; jb[t].seed = seed; jb[t].seq = seq; jb[t].t_ctg = t_ctg; jb[t].t_pos = t_pos;
		jb[t].t_strand = t_strand;
		jb[t].r0 = n_reads * t / threads; jb[t].r1 = n_reads * (t + 1) / threads;
		pthread_create(&th[t], NULL, sim_worker, &jb[t]);
	}
	for (t = 0; t < threads; t++) pthread_join(th[t], NULL);
	free(cum);
	return 0;
}
