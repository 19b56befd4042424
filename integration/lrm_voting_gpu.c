/*
 * lrm_voting_gpu.c -- the reference-side binding of sublong's voting step to libsubread_amd.so
 * (include/subread_long.h).  Compiled against the reference's own longread-one headers and linked
 * into the reference's sublong in place of its per-read loop:
 *
 *   LRMchunk_read_iteration   longread-mapping.c:1336-1357 (stock: fetch one read, vote it with
 *                             LRMdo_one_voting_read, run LRMdo_dynamic_programming_read)
 *
 * This version fetches the thread's reads in batches (the same LRMfetch_next_read, so the same
 * read numbers), votes a batch on the GPU with svg_long_vote_batch, then for each read rebuilds
 * exactly the state LRMdo_one_voting_read leaves (longread-mapping.c:552-560): the vote table's
 * used slots (pos, votes, masks, coverage; LRMconfig.h:75-86), the read text and qualities
 * reversed (LRMreverse_read_and_qual, the strand-1 pass), is_reversed = 1 -- and hands the read
 * to the reference's own LRMdo_dynamic_programming_read (copy, location sort, windows, chains,
 * gap filling, SAM/BAM record).  oracle/Makefile builds it (`make -C oracle sublong-dropin`):
 * longread-mapping.c compiled -fPIC with LRMchunk_read_iteration made weak, so
 * LRM_thread_runner's call (longread-mapping.c:406) lands here.
 *
 * Batches: up to 4096 reads or 64 Mbases per GPU call; the index handle is opened once (device
 * 0, or SVG_DEVICE) and shared by the threads under a mutex.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <pthread.h>
#include "LRMconfig.h"
#include "LRMsorted-hashtable.h"
#include "LRMfile-io.h"
#include "subread_long.h"

int LRMfetch_next_read(LRMcontext_t *context, LRMthread_context_t *thread_context, unsigned int *read_len, char *read_name,
                       char *read_text, char *qual_text, unsigned int *read_no_in_chunk);
void LRMreverse_read_and_qual(LRMcontext_t *context, LRMthread_context_t *thread_context,
                              LRMread_iteration_context_t *iteration_context);
void LRMdo_dynamic_programming_read(LRMcontext_t *context, LRMthread_context_t *thread_context,
                                    LRMread_iteration_context_t *iteration_context);
double LRMmiltime(void);

#define B_READS 4096
#define B_BASES (64u << 20)

static svg_index *g_ix;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

static svg_index *gpu_index(LRMcontext_t *context)
{
	pthread_mutex_lock(&g_mu);
	if (!g_ix) {
		const char *d = getenv("SVG_DEVICE");
		if (svg_index_open(context->index_prefix, d ? atoi(d) : 0, &g_ix)) {
			fprintf(stderr, "GPU voting unavailable: %s\n", svg_last_error());
			exit(1);
		}
	}
	pthread_mutex_unlock(&g_mu);
	return g_ix;
}

typedef struct {
	uint32_t n;
	uint64_t bases;
	char (*names)[LRMMAX_READ_NAME_LEN];
	char *text, *qual;          /* B_BASES + LRMMAX_READ_LENGTH each */
	uint64_t *off;
	uint32_t *len, *no;
} batch_t;

int LRMchunk_read_iteration(LRMcontext_t *context, int thread_id, int task)
{
	LRMthread_context_t *thread_context = context->thread_contexts + thread_id;
	LRMread_iteration_context_t *it = malloc(sizeof(LRMread_iteration_context_t));
	memset(it, 0, sizeof(LRMread_iteration_context_t));
	svg_index *ix = gpu_index(context);
	batch_t b;
	b.names = malloc(sizeof(*b.names) * B_READS);
	b.text = malloc(B_BASES + LRMMAX_READ_LENGTH);
	b.qual = malloc(B_BASES + LRMMAX_READ_LENGTH);
	b.off = malloc(8 * B_READS);
	b.len = malloc(4 * B_READS);
	b.no = malloc(4 * B_READS);
	int done = 0;
	while (!done) {
		/* the batch: LRMfetch_next_read as the stock loop calls it (read text and quality of the
		 * file, read number in the chunk) */
		b.n = 0;
		b.bases = 0;
		while (b.n < B_READS && b.bases < B_BASES) {
			unsigned int rl = 0, no = 0;
			if (LRMfetch_next_read(context, thread_context, &rl, it->read_name, b.text + b.bases, b.qual + b.bases, &no)) {
				done = 1;
				break;
			}
			memcpy(b.names[b.n], it->read_name, LRMMAX_READ_NAME_LEN);
			b.off[b.n] = b.bases;
			b.len[b.n] = rl;
			b.no[b.n] = no;
			b.bases += rl;
			b.n++;
		}
		if (!b.n) break;
		svg_long_reads R = {b.text, b.off, b.len, b.n};
		svg_long_result res;
		pthread_mutex_lock(&g_mu);
		int rc = svg_long_vote_batch(ix, &R, &res);
		pthread_mutex_unlock(&g_mu);
		if (rc) {
			fprintf(stderr, "svg_long_vote_batch failed: %s\n", svg_last_error());
			exit(1);
		}
		for (uint32_t k = 0; k < b.n; k++) {
			memcpy(it->read_name, b.names[k], LRMMAX_READ_NAME_LEN);
			memcpy(it->read_text, b.text + b.off[k], b.len[k]);
			it->read_text[b.len[k]] = 0;
			memcpy(it->qual_text, b.qual + b.off[k], b.len[k]);
			it->qual_text[b.len[k]] = 0;
			it->read_length = b.len[k];
			it->read_no_in_chunk = b.no[k];
			/* LRMdo_one_voting_read's result */
			LRMgene_vote_t *v = &it->vote_table;
			LRMinit_gene_vote(v);
			for (uint64_t s = res.vstart[k]; s < res.vstart[k + 1]; s++) {
				const svg_long_vote *x = &res.votes[s];
				const uint32_t bb = x->slot >> 16, ii = x->slot & 0xffff;
				v->pos[bb][ii] = x->pos;
				v->votes[bb][ii] = x->votes;
				v->masks[bb][ii] = x->negative ? LRMIS_NEGATIVE_STRAND : 0;
				v->coverage_start[bb][ii] = x->coverage_start;
				v->coverage_end[bb][ii] = x->coverage_end;
				v->items[bb] = (unsigned short)(ii + 1);
			}
			LRMreverse_read_and_qual(context, thread_context, it);
			it->is_reversed = 1;
			LRMdo_dynamic_programming_read(context, thread_context, it);
			if (it->read_no_in_chunk % 2000 == 0)
				LRMprintf("Processing %d-th read for task %d; used %.1f minutes\n",
				          context->all_processed_reads + it->read_no_in_chunk, task,
				          (LRMmiltime() - context->start_running_time) / 60);
		}
		svg_long_free(&res);
	}
	if (it->chain_used_gaps) LRMArrayListDestroy(it->chain_used_gaps);
	it->chain_used_gaps = NULL;
	free(it);
	free(b.names); free(b.text); free(b.qual); free(b.off); free(b.len); free(b.no);
	return 0;
}
