/*
 * TEST INFRASTRUCTURE ONLY -- never linked into the product.
 *
 * Voting-step timing harness for the CPU baseline calibration (tools/cpu_calibration.py):
 * linked into the reference aligner built from /root/reference/src (oracle/Makefile,
 * _ref/subread-align-votetime), with core.c's fetch_next_read_pair (core.c:1121-1211) made
 * weak so that this definition answers every call site (do_voting core.c:3097, iteration two
 * :2557, iteration three :2288).
 *
 * The reads are parsed once, by the reference's own parser (geinput_next_read_trim,
 * input-files.c:792), at the first call, before the clock starts; every later call hands
 * out the next read of the chunk from memory exactly as fetch_next_read_pair numbers them
 * (running_processed_reads_in_chunk under input_lock's role), with the same -S reversal.
 * The voting step's time is from the end of that parse to the last "no more reads" answer
 * of the first pass (the run_maybe_threads(STEP_VOTING) of core.c:3592: the vote, the
 * bigtable writes and the final-run tail of every read, FASTQ parsing excluded).
 * SVG_REF_VOTETIME=1 prints "SVG_REF_VOTING_S <seconds> <reads>" to stderr at exit.
 *
 * Two modes.  Default: a single chunk (reads <= reads_per_chunk), the reference's iteration two
 * and SAM as usual.  SVG_REF_CHUNK=S (the bench's cpu_baseline): reads_per_chunk is set to S at
 * the first call, so the reads go through ceil(n/S) chunks of one process (one index load), and
 * do_iteration_two -- weak in core-vt.o, answered here -- returns at once: each chunk is timed
 * from its first read handed out to its last "no more reads" answer, and
 * "SVG_REF_CHUNK_VOTING_S <chunk> <seconds> <reads>" is printed per chunk.  The vote, the
 * bigtable writes and the final-run tail are the reference's own; iteration two and SAM are not
 * run in that mode (nothing they do is on the timed path).  One-block indexes only.
 */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "subread.h"
#include "input-files.h"
#include "core.h"

struct rv_end { char **name, **text, **qual; int *len; long n, cap; };
static struct rv_end rv[2];
static pthread_mutex_t rv_mu = PTHREAD_MUTEX_INITIALIZER;
static int rv_parsed, rv_pass;
static long rv_served;
static double rv_t0, rv_t1;
// chunked vote-only mode (SVG_REF_CHUNK)
#define RV_MAX_CHUNKS 64
static long rv_chunk_size, rv_base, rv_chunk_reads[RV_MAX_CHUNKS];
static int rv_chunk = -1, rv_it2_seen;
static double rv_ct0[RV_MAX_CHUNKS], rv_ct1[RV_MAX_CHUNKS];

int ref_do_iteration_two(global_context_t *gc, thread_context_t *tc);

// run_in_thread's STEP_ITERATION_TWO call (core.c:3370): in chunked mode the chunk's voting is over
int do_iteration_two(global_context_t *gc, thread_context_t *tc)
{
	if (!rv_chunk_size) return ref_do_iteration_two(gc, tc);
	pthread_mutex_lock(&rv_mu);
	rv_it2_seen = 1;
	pthread_mutex_unlock(&rv_mu);
	return 0;
}

static double rv_now(void)
{
	struct timeval tv;
	gettimeofday(&tv, NULL);
	return tv.tv_sec + tv.tv_usec * 1e-6;
}

static void rv_parse(global_context_t *gc, gene_input_t *in, struct rv_end *e)
{
	char *name = malloc(MAX_READ_NAME_LEN + 2), *text = malloc(MAX_READ_LENGTH + 2), *qual = malloc(MAX_READ_LENGTH + 2);
	for (;;) {
		int sec = 0;
		int rl = geinput_next_read_trim(in, name, text, qual, gc->config.read_trim_5, gc->config.read_trim_3, &sec);
		if (rl <= 0) break;
		if (e->n == e->cap) {
			e->cap = e->cap ? 2 * e->cap : 1 << 16;
			e->name = realloc(e->name, e->cap * sizeof(char *));
			e->text = realloc(e->text, e->cap * sizeof(char *));
			e->qual = realloc(e->qual, e->cap * sizeof(char *));
			e->len = realloc(e->len, e->cap * sizeof(int));
		}
		e->name[e->n] = strdup(name);
		// text and quality by length: a read may hold NUL bytes (the reference works on rl bytes)
		e->text[e->n] = memcpy(malloc(rl + 1), text, rl + 1);
		e->qual[e->n] = memcpy(malloc(rl + 1), qual, rl + 1);
		e->len[e->n] = rl;
		e->n++;
	}
	free(name); free(text); free(qual);
}

int fetch_next_read_pair(global_context_t *gc, thread_context_t *tc, gene_input_t *ginp1, gene_input_t *ginp2,
                         int *read_len_1, int *read_len_2, char *read_name_1, char *read_name_2, char *read_text_1,
                         char *read_text_2, char *qual_text_1, char *qual_text_2, int remove_color_head,
                         subread_read_number_t *read_no_in_chunk)
{
	(void)tc; (void)remove_color_head;
	long num = -1, at = -1;
	pthread_mutex_lock(&rv_mu);
	if (!rv_parsed) {
		rv_parse(gc, ginp1, &rv[0]);
		if (ginp2) rv_parse(gc, ginp2, &rv[1]);
		if (ginp2 && rv[0].n != rv[1].n) { fprintf(stderr, "ref_votetime: unequal read counts\n"); exit(2); }
		const char *cs = getenv("SVG_REF_CHUNK");
		if (cs && atol(cs) > 0) {
			rv_chunk_size = atol(cs);
			if (rv_chunk_size > (long)gc->config.reads_per_chunk) { fprintf(stderr, "ref_votetime: chunk too large\n"); exit(2); }
			if ((rv[0].n + rv_chunk_size - 1) / rv_chunk_size >= RV_MAX_CHUNKS) { fprintf(stderr, "ref_votetime: too many chunks\n"); exit(2); }
			gc->config.reads_per_chunk = rv_chunk_size;
			rv_it2_seen = 1;
		} else if (rv[0].n > (long)gc->config.reads_per_chunk) { fprintf(stderr, "ref_votetime: one chunk only\n"); exit(2); }
		rv_parsed = 1;
		rv_t0 = rv_now();
	}
	if (rv_chunk_size) {
		if (rv_it2_seen) {           // the first call of a chunk's voting pass
			if (rv_chunk >= 0) rv_base += rv_chunk_reads[rv_chunk];
			rv_chunk++;
			rv_it2_seen = 0;
			rv_ct0[rv_chunk] = rv_now();
			rv_ct1[rv_chunk] = rv_ct0[rv_chunk];
		}
		if (gc->running_processed_reads_in_chunk < gc->config.reads_per_chunk &&
		    rv_base + (long)gc->running_processed_reads_in_chunk < rv[0].n) {
			num = (long)gc->running_processed_reads_in_chunk++;
			at = rv_base + num;
			rv_chunk_reads[rv_chunk] = num + 1;
		} else {
			rv_ct1[rv_chunk] = rv_now();
		}
		pthread_mutex_unlock(&rv_mu);
	} else {
		if (gc->running_processed_reads_in_chunk < gc->config.reads_per_chunk && gc->running_processed_reads_in_chunk < rv[0].n) {
			num = (long)gc->running_processed_reads_in_chunk++;
			at = num;
			if (num == 0 && rv_served) rv_pass++;   // the counter was reset: a later pass (iteration two, three)
			rv_served++;
		} else if (rv_pass == 0) {
			rv_t1 = rv_now();                       // a thread's last answer of the voting pass
		}
		pthread_mutex_unlock(&rv_mu);
	}
	if (num < 0) { *read_no_in_chunk = -1; return 1; }
	strcpy(read_name_1, rv[0].name[at]);
	memcpy(read_text_1, rv[0].text[at], rv[0].len[at] + 1);
	if (qual_text_1) memcpy(qual_text_1, rv[0].qual[at], rv[0].len[at] + 1);
	*read_len_1 = rv[0].len[at];
	if (gc->config.is_first_read_reversed) {
		reverse_read(read_text_1, *read_len_1, gc->config.space_type);
		if (qual_text_1) reverse_quality(qual_text_1, *read_len_1);
	}
	if (ginp2) {
		strcpy(read_name_2, rv[1].name[at]);
		memcpy(read_text_2, rv[1].text[at], rv[1].len[at] + 1);
		if (qual_text_2) memcpy(qual_text_2, rv[1].qual[at], rv[1].len[at] + 1);
		*read_len_2 = rv[1].len[at];
		if (gc->config.is_second_read_reversed) {
			reverse_read(read_text_2, *read_len_2, gc->config.space_type);
			if (qual_text_2) reverse_quality(qual_text_2, *read_len_2);
		}
	}
	*read_no_in_chunk = num;
	return 0;
}

__attribute__((destructor)) static void rv_report(void)
{
	const char *e = getenv("SVG_REF_VOTETIME");
	if (e && e[0] == '1' && rv_parsed) {
		if (rv_chunk_size) {
			for (int c = 0; c <= rv_chunk; c++)
				if (rv_chunk_reads[c]) fprintf(stderr, "SVG_REF_CHUNK_VOTING_S %d %.6f %ld\n", c, rv_ct1[c] - rv_ct0[c], rv_chunk_reads[c]);
		} else
			fprintf(stderr, "SVG_REF_VOTING_S %.6f %ld\n", rv_t1 - rv_t0, rv[0].n);
	}
}
