/*
 * TEST INFRASTRUCTURE ONLY -- never linked into the product.
 *
 * The svg_* entry points integration/do_voting_gpu.c calls for the vote itself
 * (svg_index_open, svg_vote_batch_packed, svg_fragile_batch, svg_last_error), answered by the
 * CPU restatement (svoracle.c) instead of the GPU.  oracle/Makefile compiles do_voting_gpu.c a second time
 * with those names mapped to the svo_dropin_* functions below and links it into the
 * reference's own subread-align / subjunc (`_ref/*-oracle-dropin`).  tests/test_dropin.py
 * runs that binary in this container (no GPU) against the stock reference: it checks the
 * binding's host logic -- chunk reading, bigtable layout, big-margin staging, text/quality
 * orientation of the post-vote tail, fragile junction voting order, block loop -- apart
 * from the kernels, whose records the GPU drop-in test (tests/test_gpu_dropin.py) then
 * checks through the same binding.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "subread_vote.h"

typedef struct svo_index svo_index;
static char err[256];
svo_index *svo_index_open(const char *prefix);
int svo_vote_batch(const svo_index *ix, const svg_params *p, const svg_reads *r1, const svg_reads *r2,
                   svg_mapping_result *out, svg_subjunc_result *jout, uint16_t *bm, int threads,
                   uint64_t *stats3);
int svo_fragile_batch(const svo_index *ix, const svg_params *p, const svg_reads *r1, const svg_reads *r2,
                      svg_fragile_result *out);

/* the fragile junction voting windows, from the restatement */
int svo_dropin_fragile_batch(svg_index *idx, const svg_params *p, const svg_reads *r1, const svg_reads *r2,
                             svg_fragile_result *out)
{
	int rc = svo_fragile_batch((const svo_index *)idx, p, r1, r2, out);
	if (rc) snprintf(err, sizeof err, "oracle fragile voting failed (%d)", rc);
	return rc;
}

const char *svo_dropin_last_error(void) { return err; }

int svo_dropin_index_open(const char *prefix, int device, svg_index **out)
{
	(void)device;
	svo_index *ix = svo_index_open(prefix);
	if (!ix) { snprintf(err, sizeof err, "cannot open index %s", prefix); return SVG_E_IO; }
	*out = (svg_index *)ix;
	return 0;
}

/* svg_index_open_devices: one restatement index per listed device */
int svo_dropin_index_open_devices(const char *prefix, const int *devices, int n, svg_index **out)
{
	for (int k = 0; k < n; k++) {
		const int rc = svo_dropin_index_open(prefix, devices[k], &out[k]);
		if (rc) return rc;
	}
	return 0;
}

/* 2-bit codes + exception mask back to characters with the same base2int code and the same
 * exception status ('.' sorts below 'G' like the code-2 exceptions, 'N' above it) */
static int unpack(const svg_packed_reads *pk, svg_reads *r, char **seq, uint64_t **off)
{
	uint64_t n = pk->n_reads, i, total = 0;
	for (i = 0; i < n; i++) total += pk->lens[i];
	*seq = malloc(total + 1);
	*off = malloc(8 * (n + 1));
	if (!*seq || !*off) return SVG_E_NOMEM;
	uint64_t at = 0;
	for (i = 0; i < n; i++) {
		uint64_t s = pk->starts ? pk->starts[i] : i * pk->stride, k;
		(*off)[i] = at;
		for (k = 0; k < pk->lens[i]; k++, s++) {
			unsigned code = (pk->bases[s / 16] >> (30 - 2 * (s % 16))) & 3;
			int x = pk->xmask && ((pk->xmask[s / 32] >> (31 - s % 32)) & 1);
			(*seq)[at++] = x ? (code == 2 ? '.' : 'N') : "AGCT"[code];
		}
	}
	r->seq = *seq; r->offsets = *off; r->lens = pk->lens; r->n_reads = n;
	return 0;
}

int svo_dropin_vote_batch_packed(svg_index *idx, const svg_params *p, const svg_packed_reads *r1,
                                 const svg_packed_reads *r2, svg_mapping_result *out, svg_subjunc_result *jout,
                                 uint16_t *big_margin)
{
	svg_reads a[2];
	char *seq[2] = {NULL, NULL};
	uint64_t *off[2] = {NULL, NULL};
	int rc = unpack(r1, &a[0], &seq[0], &off[0]);
	if (!rc && r2) rc = unpack(r2, &a[1], &seq[1], &off[1]);
	if (!rc) rc = svo_vote_batch((const svo_index *)idx, p, &a[0], r2 ? &a[1] : NULL, out, jout, big_margin, 4, NULL);
	if (rc) snprintf(err, sizeof err, "oracle vote failed (%d)", rc);
	free(seq[0]); free(seq[1]); free(off[0]); free(off[1]);
	return rc;
}
