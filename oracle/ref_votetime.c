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
 * Single chunk only (reads <= reads_per_chunk), base space only: the calibration's inputs.
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
		e->text[e->n] = strdup(text);
		e->qual[e->n] = strdup(qual);
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
	long num = -1;
	pthread_mutex_lock(&rv_mu);
	if (!rv_parsed) {
		rv_parse(gc, ginp1, &rv[0]);
		if (ginp2) rv_parse(gc, ginp2, &rv[1]);
		if (ginp2 && rv[0].n != rv[1].n) { fprintf(stderr, "ref_votetime: unequal read counts\n"); exit(2); }
		if (rv[0].n > (long)gc->config.reads_per_chunk) { fprintf(stderr, "ref_votetime: one chunk only\n"); exit(2); }
		rv_parsed = 1;
		rv_t0 = rv_now();
	}
	if (gc->running_processed_reads_in_chunk < gc->config.reads_per_chunk && gc->running_processed_reads_in_chunk < rv[0].n) {
		num = (long)gc->running_processed_reads_in_chunk++;
		if (num == 0 && rv_served) rv_pass++;   // the counter was reset: a later pass (iteration two, three)
		rv_served++;
	} else if (rv_pass == 0) {
		rv_t1 = rv_now();                       // a thread's last answer of the voting pass
	}
	pthread_mutex_unlock(&rv_mu);
	if (num < 0) { *read_no_in_chunk = -1; return 1; }
	strcpy(read_name_1, rv[0].name[num]);
	strcpy(read_text_1, rv[0].text[num]);
	if (qual_text_1) strcpy(qual_text_1, rv[0].qual[num]);
	*read_len_1 = rv[0].len[num];
	if (gc->config.is_first_read_reversed) {
		reverse_read(read_text_1, *read_len_1, gc->config.space_type);
		if (qual_text_1) reverse_quality(qual_text_1, *read_len_1);
	}
	if (ginp2) {
		strcpy(read_name_2, rv[1].name[num]);
		strcpy(read_text_2, rv[1].text[num]);
		if (qual_text_2) strcpy(qual_text_2, rv[1].qual[num]);
		*read_len_2 = rv[1].len[num];
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
	if (e && e[0] == '1' && rv_parsed)
		fprintf(stderr, "SVG_REF_VOTING_S %.6f %ld\n", rv_t1 - rv_t0, rv[0].n);
}
