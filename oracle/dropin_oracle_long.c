/*
 * TEST INFRASTRUCTURE ONLY -- never linked into the product.
 *
 * svg_long_vote_batch for integration/lrm_voting_gpu.c answered by the CPU restatement
 * (svoracle.c svo_long_vote_batch) instead of the GPU: oracle/Makefile compiles the binding a
 * second time with the svg_* names it calls mapped here and links it into the reference's own
 * sublong (`_ref/sublong-oracle-dropin`); tests/test_dropin.py runs that binary in this container
 * (no GPU) against the stock sublong -- the binding's host logic (batched fetch, vote-table
 * rebuild, text / quality orientation) apart from the kernels, which tests/test_gpu_dropin.py
 * then checks through the same binding.
 */
#include "subread_long.h"

typedef struct svo_index svo_index;
int svo_long_vote_batch(const svo_index *ix, const svg_long_reads *R, int threads, svg_long_result *out);

int svo_dropin_long_vote_batch(svg_index *idx, const svg_long_reads *R, svg_long_result *out)
{
	return svo_long_vote_batch((const svo_index *)idx, R, 1, out);
}
