/*
 * integration/do_voting_gpu.c -- the reference-side binding of include/subread_vote.h.
 *
 * What a Subread maintainer adds to subread-align / subjunc (v2.0.6) to run the voting
 * step on an MI355X: do_voting_gpu() replaces do_voting() (src/core.c:3049) for one- and
 * multi-block indexes.  tests/test_boundary_ref.py compiles it against the REFERENCE's own
 * headers, and oracle/Makefile links it into the reference's own subread-align / subjunc
 * (built from /root/reference/src, `make -C oracle dropin`), whose run_in_thread call to
 * do_voting (core.c:3366-3368) then lands here; tests/test_gpu_dropin.py compares the SAM,
 * VCF and junction BED of that binary with the stock reference's, byte for byte.
 *
 *   svg_attach           once, after load_global_context (core.c:4013) has the index prefix
 *   svg_attach_devices   the same for several GPUs: one handle (a full index replica) per device;
 *                        each chunk's reads are then split into contiguous ranges, one per handle,
 *                        voted by one host thread per handle into the one bigtable
 *   do_voting_gpu        per chunk and index block, from ONE host thread per GPU
 *                        (run_in_thread, core.c:3366)
 *   do_voting_gpu_mt     the same from each of the run's -T threads: thread 0 reads and votes
 *                        the chunk, every thread does the per-read host work of its slice
 *
 * The chunk's reads come from fetch_next_read_pair (core.c:1121) exactly as do_voting
 * reads them -- that function already applies the -S reversal (core.c:1186-1198), so the
 * library is told not to reverse again (reverse_r1 = reverse_r2 = 0).  Reads are 2-bit
 * packed on the host (svg_pack_reads) and voted with svg_vote_batch_packed straight into
 * the chunk's bigtable (core-bigtable.c:84-131).  Subjunc reads > 160 bp also get their
 * fragile junction voting windows (core_fragile_junction_voting, core.c:3138-3142 ->
 * core-junction.c:5151-5422: gehash_go_q windows, select_best_vote, the best matching halves,
 * the donor test) from the GPU in the same block-0 run (svg_fragile_batch, every block's
 * windows).  The per-read host work of do_voting then runs in do_voting's order in the library
 * (include/subread_events.h), each thread's slice of the chunk into that thread's event table:
 *   - fragile windows -> events (core-junction.c:5211-5419), each index block's windows in that
 *     block's run (svg_events_add_windows);
 *   - the final voting run: find_new_indels / find_new_junctions per record (core.c:3240-3290),
 *     after the read's last-block windows (svg_events_add_batch2).
 * The library's table starts as an exact copy of the run's table (events and site lists,
 * svg_events_load_sites) and its changes come back into it (event_to_ref, put_new_event).  The
 * reference's functions (fragile_window_events_ref, tail_ref) stay for what the library does not
 * cover, and every stage says which implementation ran (SVG_DROPIN_STAGES at exit;
 * SVG_REQUIRE_LIBRARY=1 makes a use of the reference's function an error).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <ctype.h>
#include <unistd.h>
#include "subread.h"
#include "core.h"
#include "core-indel.h"
#include "core-junction.h"
#include "input-files.h"
#include "gene-algorithms.h"
#include "subread_vote.h"
#include "subread_realign.h"

/* defined in core.c (non-static there, not declared in a header) */
int fetch_next_read_pair(global_context_t *global_context, thread_context_t *thread_context, gene_input_t *ginp1,
                         gene_input_t *ginp2, int *read_len_1, int *read_len_2, char *read_name_1, char *read_name_2,
                         char *read_text_1, char *read_text_2, char *qual_text_1, char *qual_text_2,
                         int remove_color_head, subread_read_number_t *read_no_in_chunk);
void init_chunk_scanning_parameters(global_context_t *global_context, thread_context_t *thread_context,
                                    gene_input_t **ginp1, gene_input_t **ginp2);
int locate_current_value_index(global_context_t *global_context, thread_context_t *thread_context,
                               mapping_result_t *result, int rlen);
int has_better_mapping(global_context_t *global_context, thread_context_t *thread_context,
                       subread_read_number_t current_read_number, int is_second_read, int this_aln_id);
int find_subread_end(int len, int TOTAL_SUBREADS, int subread);   /* input-files.c:1371 */
void set_insertion_sequence(global_context_t *gc, thread_context_t *tc, char **binary_bases, char *read_text,
                            int insertions);                     /* core-indel.c:1479 */

/*
 * Which implementation answered each stage (printed at exit by svg_sam_finish as one
 * SVG_DROPIN_STAGES line): the library -- the GPU vote and fragile windows, the host-C event stage,
 * anti-supporting read scan, remove_neighbour and iteration two -- or the reference's own function
 * this binding falls back to for a configuration the library does not cover.  With
 * SVG_REQUIRE_LIBRARY=1 a fallback ends the run at once (exit status 3) with its reason.
 */
enum { ST_VOTE, ST_FRAGILE, ST_EVENTS, ST_ANTI, ST_RN, ST_IT2, ST_N };
static const char *const svg_stage_name[ST_N] = {"vote", "fragile", "events", "anti_support", "remove_neighbour", "iteration_two"};
static long svg_stage_n[ST_N][2];   /* [stage][0: library, 1: the reference's function] */

static void svg_stages_print(FILE *fp)
{
	fprintf(fp, "SVG_DROPIN_STAGES");
	for (int k = 0; k < ST_N; k++)
		fprintf(fp, " %s=library:%ld,reference:%ld", svg_stage_name[k], __atomic_load_n(&svg_stage_n[k][0], __ATOMIC_RELAXED),
		        __atomic_load_n(&svg_stage_n[k][1], __ATOMIC_RELAXED));
	fprintf(fp, "\n");
}

/* one run of stage `st`: by the library (why == NULL) or by the reference's function, for `why` */
static void svg_stage(int st, const char *why)
{
	__atomic_fetch_add(&svg_stage_n[st][why ? 1 : 0], 1, __ATOMIC_RELAXED);
	if (!why) return;
	const char *req = getenv("SVG_REQUIRE_LIBRARY");
	if (getenv("SVG_REF_TIMING") || (req && req[0] == '1'))
		fprintf(stderr, "SVG_DROPIN_FALLBACK %s: the reference's function (%s)\n", svg_stage_name[st], why);
	if (req && req[0] == '1') {
		fprintf(stderr, "SVG_REQUIRE_LIBRARY=1: stage %s fell back to the reference's function: %s\n", svg_stage_name[st], why);
		svg_stages_print(stderr);
		fflush(NULL);
		_exit(3);
	}
}

/* The handles: svg_ix[0 .. svg_nix-1], one per device (svg_attach_devices), each with a full index
 * replica in its HBM.  The reads of a chunk are independent, so handle k votes the k-th contiguous
 * range of them straight into the bigtable rows of those reads -- the fan-out of run_maybe_threads
 * (core.c:3379-3461), with GPUs in the role of its threads; no exchange between devices. */
#define SVG_MAX_DEV 16
static svg_index *svg_ix[SVG_MAX_DEV];
static int svg_nix;
static double svg_t_open;      /* SVG_REF_TIMING: svg_index_open of every handle (the index files into HBM) */
static pthread_mutex_t svg_sam_mu_init = PTHREAD_MUTEX_INITIALIZER;   /* one-time setup of the shared state */
/* the handles are open before the first vote: the drop-in opens them on a thread of its own
 * (overlapping the first chunk's read, do_voting below); a host that calls svg_attach itself has
 * them already */
#ifdef SVG_DROPIN_DO_VOTING
static int svg_open_join(void);
#else
static int svg_open_join(void) { return svg_nix > 0 ? 0 : 1; }
#endif

typedef struct { const char *prefix; int device; svg_index *ix; int rc; char err[256]; } svg_opener;
static void *svg_opener_run(void *v)
{
	svg_opener *o = v;
	o->rc = svg_index_open(o->prefix, o->device, &o->ix);
	if (o->rc) snprintf(o->err, sizeof o->err, "%s", svg_last_error());
	return NULL;
}

int svg_attach_devices(global_context_t *gc, const int *devices, int n)
{
	char prefix[MAX_FILE_NAME_LENGTH + 1];
	int k, rc = 0;
	if (n < 1 || n > SVG_MAX_DEV) {
		SUBREADprintf("GPU voting: %d devices (1 .. %d)\n", n, SVG_MAX_DEV);
		return 1;
	}
	snprintf(prefix, sizeof prefix, "%s", gc->config.index_prefix);
	const double t0 = miltime();
	if (n == 1) {
		svg_opener op = {prefix, devices[0], NULL, 0, ""};
		svg_opener_run(&op);
		rc = op.rc;
		if (rc) SUBREADprintf("GPU voting unavailable on device %d: %s\n", devices[0], op.err);
		else svg_ix[0] = op.ix;
	} else {
		/* one replica per device from ONE read of the index files: the .tab is walked and staged once
		 * and every staged run is copied to every device (svg_index_open_devices) */
		rc = svg_index_open_devices(prefix, devices, n, svg_ix);
		if (rc) {
			SUBREADprintf("GPU voting unavailable on devices");
			for (k = 0; k < n; k++) SUBREADprintf(" %d", devices[k]);
			SUBREADprintf(": %s\n", svg_last_error());
			for (k = 0; k < n; k++) svg_ix[k] = NULL;
		}
	}
	if (!rc) svg_nix = n;
	svg_t_open += miltime() - t0;
	return rc;
}

int svg_attach(global_context_t *gc, int device)
{
	return svg_attach_devices(gc, &device, 1);
}

static void svg_fill_params(global_context_t *gc, svg_params *p)
{
	svg_params_default(p, gc->config.do_breakpoint_detection ? SVG_PROGRAM_SUBJUNC : SVG_PROGRAM_ALIGN,
	                   gc->input_reads.is_paired_end_reads);
	p->total_subreads = gc->config.total_subreads;
	p->min_votes_first = gc->config.minimum_subread_for_first_read;
	p->min_votes_second = gc->config.minimum_subread_for_second_read;
	p->max_indel_length = gc->config.max_indel_length;
	p->multi_best = gc->config.multi_best_reads;
	p->top_scores = gc->config.top_scores;
	p->max_vote_simples = gc->config.max_vote_simples;
	p->max_vote_combinations = gc->config.max_vote_combinations;
	p->max_vote_number_cutoff = gc->config.max_vote_number_cutoff;
	p->min_pair_distance = gc->config.minimum_pair_distance;
	p->max_pair_distance = gc->config.maximum_pair_distance;
	/* fetch_next_read_pair has already reversed the reads that -S asks for */
	p->reverse_r1 = 0;
	p->reverse_r2 = 0;
	p->do_breakpoint_detection = gc->config.do_breakpoint_detection;
	p->do_big_margin_filtering_for_junctions = gc->config.do_big_margin_filtering_for_junctions;
	p->big_margin_record_size = gc->config.big_margin_record_size;
	p->maximum_intron_length = gc->config.maximum_intron_length;
	p->prefer_donor_receptor_junctions = gc->config.prefer_donor_receptor_junctions;
	p->check_donor_at_junctions = gc->config.check_donor_at_junctions;
	p->max_insertion_at_junctions = gc->config.max_insertion_at_junctions;
	p->more_accurate_fusions = gc->config.more_accurate_fusions;
}

/* the chunk's reads as fetch_next_read_pair hands them to do_voting: text, names, qualities */
typedef struct {
	char *text[2], *qual[2];
	char *names[2];                    /* read names back to back, NUL-terminated; read r's at noff[e][r] */
	uint16_t *len[2];
	uint64_t *off[2], *noff[2];
	uint64_t n, cap, bytes[2], bcap[2], nbytes[2], ncap[2];
} svg_chunk_reads;

static inline char *chunk_name(const svg_chunk_reads *c, int e, uint64_t r) { return c->names[e] + c->noff[e][r]; }

static int chunk_push(svg_chunk_reads *c, int e, const char *text, const char *qual, const char *name, int len)
{
	if (c->bytes[e] + len + 1 > c->bcap[e]) {
		c->bcap[e] = (c->bcap[e] + len + 1) * 2;
		c->text[e] = realloc(c->text[e], c->bcap[e]);
		c->qual[e] = realloc(c->qual[e], c->bcap[e]);
		if (!c->text[e] || !c->qual[e]) return -1;
	}
	memcpy(c->text[e] + c->bytes[e], text, len);
	memcpy(c->qual[e] + c->bytes[e], qual, len);
	c->off[e][c->n] = c->bytes[e];
	c->len[e][c->n] = (uint16_t)len;
	{
		const size_t nl = strnlen(name, MAX_READ_NAME_LEN);
		if (c->nbytes[e] + nl + 1 > c->ncap[e]) {
			c->ncap[e] = (c->ncap[e] + nl + 1) * 2 + 4096;
			c->names[e] = realloc(c->names[e], c->ncap[e]);
			if (!c->names[e]) return -1;
		}
		memcpy(c->names[e] + c->nbytes[e], name, nl);
		c->names[e][c->nbytes[e] + nl] = 0;
		c->noff[e][c->n] = c->nbytes[e];
		c->nbytes[e] += nl + 1;
	}
	c->bytes[e] += len;
	return 0;
}

static void chunk_free(svg_chunk_reads *c)
{
	int e;
	for (e = 0; e < 2; e++) {
		free(c->text[e]); free(c->qual[e]); free(c->names[e]); free(c->len[e]); free(c->off[e]); free(c->noff[e]);
	}
}

static void fqb_begin(gene_input_t *ginp1, gene_input_t *ginp2);
static void fqb_end(void);

/* 1. the chunk's reads, in chunk read-number order (one thread: numbers are sequential); plain
 * FASTQ input is read in bulk meanwhile (fqb_begin / fqb_end, below) */
static int read_chunk(global_context_t *gc, thread_context_t *tc, int ends, svg_chunk_reads *c)
{
	gene_input_t *ginp1 = NULL, *ginp2 = NULL;
	char text[2][MAX_READ_LENGTH + 1], qual[2][MAX_READ_LENGTH + 1], name[2][MAX_READ_NAME_LEN + 1];
	int len[2] = {0, 0}, e, rc = 0;
	subread_read_number_t rno = 0;
	init_chunk_scanning_parameters(gc, tc, &ginp1, &ginp2);
	fqb_begin(ginp1, ginp2);
	for (;;) {
		fetch_next_read_pair(gc, tc, ginp1, ginp2, &len[0], &len[1], name[0], name[1], text[0], text[1], qual[0],
		                     qual[1], 1, &rno);
		if (rno < 0) break;
		if ((uint64_t)rno != c->n) {
			SUBREADprintf("do_voting_gpu: read numbers are not sequential (%lld after %llu reads)\n",
			              (long long)rno, (unsigned long long)c->n);
			rc = 1;
			break;
		}
		if (c->n == c->cap) {
			c->cap = c->cap ? 2 * c->cap : 1 << 16;
			for (e = 0; e < ends; e++) {
				c->len[e] = realloc(c->len[e], c->cap * sizeof(uint16_t));
				c->off[e] = realloc(c->off[e], c->cap * sizeof(uint64_t));
				c->noff[e] = realloc(c->noff[e], c->cap * sizeof(uint64_t));
				if (!c->len[e] || !c->off[e] || !c->noff[e]) rc = 1;
			}
			if (rc) break;
		}
		for (e = 0; e < ends && !rc; e++)
			if (chunk_push(c, e, text[e], qual[e], name[e], len[e])) rc = 1;
		if (rc) break;
		c->n++;
	}
	fqb_end();
	return rc;
}

/* one handle's share of a chunk: reads [r0, r1) of the packed chunk, records into their rows */
typedef struct {
	svg_index *ix;
	const svg_params *p;
	int ends;
	svg_packed_reads pk[2];
	svg_mapping_result *out;
	svg_subjunc_result *jout;
	uint16_t *bm;
	int rc;
	char err[256];
} svg_share;

static void *svg_share_run(void *v)
{
	svg_share *s = v;
	s->rc = svg_vote_batch_packed(s->ix, s->p, &s->pk[0], s->ends == 2 ? &s->pk[1] : NULL, s->out, s->jout, s->bm);
	if (s->rc) snprintf(s->err, sizeof s->err, "%s", svg_last_error());
	return NULL;
}

/* the big-margin records of the chunk as the vote wrote them (read, end, SVG_BIG_MARGIN_WORDS), kept
 * for the event stage of the final run; NULL without big-margin filtering */
static uint16_t *svg_bm;

/* 2. the chunk's packed reads voted into the bigtable: one call, or with several handles one
 * contiguous range of reads per handle, each from its own host thread */
static int vote_chunk(global_context_t *gc, int ends, const svg_chunk_reads *c)
{
	svg_params p;
	svg_fill_params(gc, &p);
	svg_packed_reads pk[2];
	uint32_t *bases[2] = {NULL, NULL}, *xmask[2] = {NULL, NULL};
	uint64_t *starts[2] = {NULL, NULL};
	uint16_t *bm = NULL;
	int rc = 0, e;
	for (e = 0; e < ends && !rc; e++) {
		svg_reads r = {c->text[e], c->off[e], c->len[e], c->n};
		bases[e] = malloc(4 * (c->bytes[e] / 16 + 1));
		xmask[e] = malloc(4 * (c->bytes[e] / 32 + 1));
		starts[e] = malloc(8 * (c->n + 1));
		if (!bases[e] || !xmask[e] || !starts[e]) { rc = SVG_E_NOMEM; break; }
		int64_t nx = svg_pack_reads(&r, 0, bases[e], xmask[e], starts[e], gc->config.all_threads);
		if (nx < 0) { rc = (int)nx; break; }
		svg_packed_reads q = {bases[e], nx ? xmask[e] : NULL, starts[e], 0, c->len[e], c->n};
		pk[e] = q;
	}
	/* big-margin records live inside each bigtable_cached_result_t (core.h:453), not in one
	 * array: the library writes them to a staging array, copied into the entries below */
	if (!rc && p.do_big_margin_filtering_for_junctions) {
		bm = malloc(sizeof(uint16_t) * SVG_BIG_MARGIN_WORDS * ends * (c->n + 1));
		if (!bm) rc = SVG_E_NOMEM;
	}
	if (!rc) {
		svg_mapping_result *out = (svg_mapping_result *)_global_retrieve_alignment_ptr(gc, 0, 0, 0);
		svg_subjunc_result *jout = p.do_breakpoint_detection ? (svg_subjunc_result *)_global_retrieve_subjunc_ptr(gc, 0, 0, 0) : NULL;
		const uint64_t per = (uint64_t)ends * (uint64_t)p.multi_best;
		int nh = svg_nix, k;
		if ((uint64_t)nh > c->n) nh = c->n ? (int)c->n : 1;
		svg_share sh[SVG_MAX_DEV];
		pthread_t th[SVG_MAX_DEV];
		int started[SVG_MAX_DEV];
		memset(sh, 0, sizeof sh);
		for (k = 0; k < nh; k++) {
			const uint64_t r0 = c->n * (uint64_t)k / (uint64_t)nh, r1 = c->n * (uint64_t)(k + 1) / (uint64_t)nh;
			int e;
			sh[k].ix = svg_ix[k];
			sh[k].p = &p;
			sh[k].ends = ends;
			for (e = 0; e < ends; e++) {
				/* the range's starts / lengths / count; the packed codes and the exception mask stay
				 * shared (starts are absolute base offsets) */
				sh[k].pk[e] = pk[e];
				sh[k].pk[e].starts = pk[e].starts + r0;
				sh[k].pk[e].lens = pk[e].lens + r0;
				sh[k].pk[e].n_reads = r1 - r0;
			}
			sh[k].out = out + r0 * per;
			sh[k].jout = jout ? jout + r0 * per : NULL;
			sh[k].bm = bm ? bm + r0 * ends * SVG_BIG_MARGIN_WORDS : NULL;
			started[k] = 0;
		}
		if (nh == 1) svg_share_run(&sh[0]);
		else {
			for (k = 0; k < nh; k++) started[k] = pthread_create(&th[k], NULL, svg_share_run, &sh[k]) == 0;
			for (k = 0; k < nh; k++) {
				if (started[k]) pthread_join(th[k], NULL);
				else svg_share_run(&sh[k]);
			}
		}
		for (k = 0; k < nh && !rc; k++)
			if (sh[k].rc) {
				rc = sh[k].rc;
				SUBREADprintf("svg_vote_batch_packed (handle %d): %s\n", k, sh[k].err);
			}
	}
	if (!rc && bm) {
		uint64_t r;
		int words = gc->config.big_margin_record_size;
		for (r = 0; r < c->n; r++)
			for (e = 0; e < ends; e++)
				memcpy(_global_retrieve_big_margin_ptr(gc, r, e), bm + (r * ends + e) * SVG_BIG_MARGIN_WORDS,
				       sizeof(uint16_t) * words);
	}
	for (e = 0; e < 2; e++) { free(bases[e]); free(xmask[e]); free(starts[e]); }
	free(svg_bm);
	svg_bm = bm;
	return rc;
}

/*
 * The reference-function fallback of the event stage for one fragile-voting window that
 * svg_fragile_batch voted on the GPU: the tail of core_fragile_junction_voting
 * (core-junction.c:5211-5419) with the reference's own core_dynamic_align / local_add_indel_event /
 * search_event / put_new_event.  `in` is the window's text (NUL-terminated), as
 * core_fragile_junction_voting's InBuff.  (The library's is svg_events_add_windows / _add_batch2.)
 */
static void fragile_window_events_ref(global_context_t *gc, thread_context_t *tc, const svg_fragile_window *W,
                                      const svg_fragile_slot *slots, char *in, char *rname)
{
	indel_context_t *ic = (indel_context_t *)gc->module_contexts[MODULE_INDEL_ID];
	indel_thread_context_t *itc = tc ? (indel_thread_context_t *)tc->module_thread_contexts[MODULE_INDEL_ID] : NULL;
	HashTable *event_table = itc ? itc->event_entry_table : ic->event_entry_table;
	const int gap = gc->current_index->index_gap, read_len = W->length;
	unsigned q;
	for (q = 0; q < W->n_slots; q++) {
		const svg_fragile_slot *S = &slots[W->first_slot + q];
		int kk, last_indel = 0, last_correct_subread = 0;
		for (kk = 0; S->rec[kk] && kk < MAX_INDEL_SECTIONS; kk += 3) {
			char movement_buffer[MAX_READ_LENGTH * 10 / 7];
			int last_event_id = -1, x1, dyna_steps;
			int indels = S->rec[kk + 2] - last_indel;
			if (indels == 0) continue;
			int next_correct_subread = S->rec[kk] - 1;
			int last_correct_base = find_subread_end(read_len, gc->config.total_subreads, last_correct_subread) - 9;
			int first_correct_base = find_subread_end(read_len, gc->config.total_subreads, next_correct_subread) - 16 + 9;
			first_correct_base = min(first_correct_base + 10, read_len);
			last_correct_base = max(0, last_correct_base);
			last_correct_base = min(read_len - 1, last_correct_base);
			dyna_steps = core_dynamic_align(gc, tc, in + last_correct_base, first_correct_base - last_correct_base,
			                                S->position + last_correct_base + last_indel, movement_buffer, indels, rname);
			movement_buffer[dyna_steps] = 0;
			unsigned int cursor_on_chromosome = S->position + last_correct_base + last_indel, cursor_on_read = last_correct_base;
			int last_mv = 0, is_in_indel = 0, current_indel_len = 0, total_mismatch = 0;
			unsigned int indel_left_boundary = 0;
			for (x1 = 0; x1 < dyna_steps; x1++) if (movement_buffer[x1] == 3) total_mismatch++;
			if (total_mismatch < 2 || (gc->config.maximise_sensitivity_indel && total_mismatch <= 2))
				for (x1 = 0; x1 < dyna_steps; x1++) {
					int mv = movement_buffer[x1];
					if (last_mv != mv) {
						if ((mv == 1 || mv == 2) && !is_in_indel) {
							indel_left_boundary = cursor_on_chromosome;
							is_in_indel = 1;
							current_indel_len = 0;
						} else if (is_in_indel && (mv == 0 || mv == 3)) {
							/* (the ambiguity count core-junction.c:5283-5292 computes is unused) */
							if (abs(current_indel_len) <= gc->config.max_indel_length) {
								chromosome_event_t *new_event = local_add_indel_event(gc, tc, event_table,
								        in + cursor_on_read + min(0, current_indel_len), indel_left_boundary - 1, current_indel_len, 1, 0, 0, NULL);
								if (last_event_id >= 0 && new_event) {
									chromosome_event_t *event_space = itc ? itc->event_space_dynamic : ic->event_space_dynamic;
									chromosome_event_t *last_event = event_space + last_event_id;
									int dist = new_event->event_small_side - last_event->event_large_side + 1;
									new_event->connected_previous_event_distance = dist;
									last_event->connected_next_event_distance = dist;
								}
								last_event_id = new_event ? new_event->global_event_id : -1;
							}
						}
						if (mv == 0 || mv == 3) is_in_indel = 0;
					}
					if (is_in_indel && mv == 1) current_indel_len += 1;
					if (is_in_indel && mv == 2) current_indel_len -= 1;
					if (mv == 1 || mv == 3 || mv == 0) cursor_on_chromosome++;
					if (mv == 2 || mv == 3 || mv == 0) cursor_on_read++;
					last_mv = mv;
				}
			/* indel_recorder[i + 1] with the voting loop's i (== GENE_SLIDING_STEP) */
			last_correct_subread = S->rec[gap + 1] - 1;
		}
	}
	if (W->junction) {
		chromosome_event_t *search_return[MAX_EVENT_ENTRIES_PER_SITE], *found = NULL;
		chromosome_event_t *event_space = itc ? itc->event_space_dynamic : ic->event_space_dynamic;
		int kx1, found_events = search_event(gc, event_table, event_space, W->small_side, EVENT_SEARCH_BY_SMALL_SIDE,
		                                     CHRO_EVENT_TYPE_JUNCTION | CHRO_EVENT_TYPE_FUSION, search_return);
		for (kx1 = 0; kx1 < found_events; kx1++)
			if (search_return[kx1]->event_large_side == W->large_side) { found = search_return[kx1]; break; }
		if (found) found->supporting_reads++;
		else {
			int event_no = itc ? itc->total_events++ : ic->total_events++;
			event_space = reallocate_event_space(gc, tc, event_no);
			chromosome_event_t *new_event = event_space + event_no;
			memset(new_event, 0, sizeof(chromosome_event_t));
			new_event->event_small_side = W->small_side;
			new_event->event_large_side = W->large_side;
			new_event->is_negative_strand = !W->gtag;
			new_event->event_type = CHRO_EVENT_TYPE_JUNCTION;
			new_event->supporting_reads = 1;
			new_event->indel_length = 0;
			put_new_event(event_table, new_event, event_no);
		}
	}
}

/* svg_fragile_batch's result for the chunk being voted: made in the first block's run, used by
 * every block's run, freed after the final one */
static svg_fragile_result svg_frag;

/* the chunk of the current run, shared by the run's threads (read and voted by thread 0) */
static svg_chunk_reads svg_chunk;
/* SVG_REF_TIMING=1: the voting phase's own split, cumulative over runs, printed by svg_sam_finish
 * beside the reference's clocks (oracle/ref_dump_hook.c): reading the chunk, the vote call
 * (packing + GPU), fragile voting, and the per-read tail (slowest thread of each run) */
static double svg_t_read, svg_t_vote, svg_t_frag, svg_t_tail;
static double svg_t_realign;   /* the library's iteration two (drop-in build), cumulative */
static double svg_t_anti;      /* the library's anti-supporting read scan (drop-in build), cumulative */
/* where the time between the voting step and iteration two goes (SVG_REF_TIMING): from the end of the
 * last voting run to the anti-supporting read scan (the reference's table merge, core.c:3452), and
 * from remove_neighbour's end to iteration two (the rewind, core.c:3631-3640) */
static double svg_t_mark, svg_t_to_anti, svg_t_to_it2;
static uint64_t *svg_win;       /* svg_win[r] .. svg_win[r+1]: read r's fragile windows in this block */

static const char *svg_ev_why;
static const char *svg_events_unsupported(global_context_t *gc);

/* thread 0 (or the only thread): the chunk's reads, the GPU vote (first block's run: every block),
 * the fragile windows, and the per-read index of this block's windows */
static int vote_stage(global_context_t *gc, thread_context_t *tc)
{
	int ends = 1 + gc->input_reads.is_paired_end_reads, rc;
	memset(&svg_chunk, 0, sizeof svg_chunk);
	svg_chunk_reads *c = &svg_chunk;
	double t0 = miltime();
	rc = read_chunk(gc, tc, ends, c);
	svg_t_read += miltime() - t0;
	/* the handles' opener thread is joined whatever the read returned (it may be inside HIP
	 * initialisation or an upload; nothing may leave with it running) */
	const int open_rc = svg_open_join();
	if (!rc && open_rc) {
		SUBREADprintf("GPU voting unavailable\n");
		rc = 1;
	}
	/* a multi-block index: the library votes every block (all resident in HBM) in the first
	 * block's run of read_chunk_circles (core.c:3567-3613); the later runs re-read the chunk
	 * for the per-block host work */
	if (!rc && c->n && gc->current_index_block_number == 0) {
		t0 = miltime();
		rc = vote_chunk(gc, ends, c);
		svg_t_vote += miltime() - t0;
		if (!rc) svg_stage(ST_VOTE, NULL);
		t0 = miltime();
		/* fragile junction voting of every block, on the GPU (subjunc reads > 160 bp) */
		svg_fragile_free(&svg_frag);
		if (!rc && gc->config.do_breakpoint_detection) {
			svg_params p;
			svg_fill_params(gc, &p);
			svg_reads a1 = {c->text[0], c->off[0], c->len[0], c->n}, a2 = {c->text[1], c->off[1], c->len[1], c->n};
			rc = svg_fragile_batch(svg_ix[0], &p, &a1, ends == 2 ? &a2 : NULL, &svg_frag);
			if (rc) SUBREADprintf("svg_fragile_batch: %s\n", svg_last_error());
			else svg_stage(ST_FRAGILE, NULL);
		}
		svg_t_frag += miltime() - t0;
	}
	/* the event stage of this run: the library's, unless the configuration is one it does not cover */
	svg_ev_why = svg_events_unsupported(gc);
	/* this block's fragile windows are in (read, strand, end, window) order: read r's are
	 * svg_win[r] .. svg_win[r+1]-1 */
	free(svg_win);
	svg_win = calloc(c->n + 2, sizeof(uint64_t));
	if (!svg_win) return 1;
	uint64_t fw = 0;
	while (fw < svg_frag.n_windows && svg_frag.windows[fw].block < gc->current_index_block_number) fw++;
	for (uint64_t r = 0; r <= c->n; r++) {
		svg_win[r] = fw;
		while (fw < svg_frag.n_windows && svg_frag.windows[fw].block == gc->current_index_block_number &&
		       svg_frag.windows[fw].read == (uint32_t)r)
			fw++;
	}
	return rc;
}

/* the reference-function fallback of the event stage: do_voting's per-read host work for reads
 * [r0, r1) of the chunk, in its order, into tc's event tables (the reference's threads each fill
 * their own, merged by finalise_indel_and_junction_thread, core.c:3452) */
static void tail_stage_ref(global_context_t *gc, thread_context_t *tc, uint64_t r0, uint64_t r1)
{
	const svg_chunk_reads *c = &svg_chunk;
	int ends = 1 + gc->input_reads.is_paired_end_reads, e;
	/* do_voting's per-run state (core.c:3081-3089) */
	if (tc) tc->current_value_index = gc->current_value_index;
	int need_junction_step = gc->config.do_breakpoint_detection || gc->config.do_fusion_detection || gc->config.do_long_del_detection;
	char text[MAX_READ_LENGTH + 1], qual[MAX_READ_LENGTH + 1];
	subread_read_number_t r;
	for (r = (subread_read_number_t)r0; r < (subread_read_number_t)r1; r++) {
		/* core_fragile_junction_voting (core.c:3138-3142) of this read: its windows in this block,
		 * strand 0 on the fetched text, strand 1 on its reverse_read, R1 then R2 -- voted on the
		 * GPU (svg_fragile_batch), their events made here */
		uint64_t fw;
		for (fw = svg_win[r]; fw < svg_win[r + 1]; fw++) {
			const svg_fragile_window *W = &svg_frag.windows[fw];
			char in[MAX_READ_LENGTH + 1];
			int rl = c->len[W->end][r];
			memcpy(text, c->text[W->end] + c->off[W->end][r], rl);
			text[rl] = 0;
			if (W->strand) reverse_read(text, rl, gc->config.space_type);
			memcpy(in, text + W->start, W->length);
			in[W->length] = 0;
			fragile_window_events_ref(gc, tc, W, svg_frag.slots, in, chunk_name(c, 0, r));
		}
		if (!gc->is_final_voting_run) continue;
		/* the final-voting-run block (core.c:3240-3290) */
		for (e = 0; e < ends; e++) {
			/* do_voting leaves the text reversed once (core.c:3229-3234) and the quality as fetched;
			 * the tail starts from that state (read_1_reversed = 1) and reverses both together when a
			 * record's strand needs it, so text and quality stay in opposite orientations, as there */
			int has_reversed = 1;
			int rl = c->len[e][r];
			memcpy(text, c->text[e] + c->off[e][r], rl);
			memcpy(qual, c->qual[e] + c->off[e][r], rl);
			text[rl] = qual[rl] = 0;
			reverse_read(text, rl, gc->config.space_type);
			char *rn = chunk_name(c, e, r);
			int b;
			for (b = 0; b < gc->config.multi_best_reads; b++) {
				mapping_result_t *cur = _global_retrieve_alignment_ptr(gc, r, e, b);
				if (cur->selected_votes < 1) continue;
				int should = (cur->result_flags & CORE_IS_NEGATIVE_STRAND) ? 1 : 0;
				if (should != has_reversed) {
					has_reversed = !has_reversed;
					reverse_read(text, rl, gc->config.space_type);
					reverse_quality(qual, rl);
				}
				gene_value_index_t *saved = tc ? tc->current_value_index : gc->current_value_index;
				locate_current_value_index(gc, tc, cur, rl);
				if (!has_better_mapping(gc, tc, r, e, b)) find_new_indels(gc, tc, r, rn, text, qual, rl, e, b);
				if (need_junction_step) find_new_junctions(gc, tc, r, rn, text, qual, rl, e, b);
				if (tc) tc->current_value_index = saved;
				else gc->current_value_index = saved;
			}
		}
	}
}


/* chromosome_event_t <-> svg_event: every field but the inserted bases' pointer and the id */
static void event_to_svg(const chromosome_event_t *e, svg_event *o)
{
	memset(o, 0, sizeof *o);
	o->small_side = e->event_small_side;
	o->large_side = e->event_large_side;
	o->indel_length = e->indel_length;
	o->junction_flanking_left = e->junction_flanking_left;
	o->junction_flanking_right = e->junction_flanking_right;
	o->indel_at_junction = e->indel_at_junction;
	o->is_negative_strand = e->is_negative_strand;
	o->is_strand_jumped = e->is_strand_jumped;
	o->is_donor_found_or_annotation = e->is_donor_found_or_annotation;
	o->small_side_increasing_coordinate = e->small_side_increasing_coordinate;
	o->large_side_increasing_coordinate = e->large_side_increasing_coordinate;
	o->connected_next_event_distance = e->connected_next_event_distance;
	o->connected_previous_event_distance = e->connected_previous_event_distance;
	o->supporting_reads = e->supporting_reads;
	o->anti_supporting_reads = e->anti_supporting_reads;
	o->final_counted_reads = e->final_counted_reads;
	o->final_reads_mismatches = e->final_reads_mismatches;
	o->event_type = e->event_type;
	o->critical_read_id = e->critical_read_id;
	o->event_quality = e->event_quality;
	o->critical_supporting_reads = e->critical_supporting_reads;
}

static void event_to_ref(const svg_event *o, chromosome_event_t *e)
{
	e->event_small_side = o->small_side;
	e->event_large_side = o->large_side;
	e->indel_length = o->indel_length;
	e->junction_flanking_left = o->junction_flanking_left;
	e->junction_flanking_right = o->junction_flanking_right;
	e->indel_at_junction = o->indel_at_junction;
	e->is_negative_strand = o->is_negative_strand;
	e->is_strand_jumped = o->is_strand_jumped;
	e->is_donor_found_or_annotation = o->is_donor_found_or_annotation;
	e->small_side_increasing_coordinate = o->small_side_increasing_coordinate;
	e->large_side_increasing_coordinate = o->large_side_increasing_coordinate;
	e->connected_next_event_distance = o->connected_next_event_distance;
	e->connected_previous_event_distance = o->connected_previous_event_distance;
	e->supporting_reads = o->supporting_reads;
	e->anti_supporting_reads = o->anti_supporting_reads;
	e->final_counted_reads = o->final_counted_reads;
	e->final_reads_mismatches = o->final_reads_mismatches;
	e->event_type = o->event_type;
	e->critical_read_id = o->critical_read_id;
	e->event_quality = o->event_quality;
	e->critical_supporting_reads = o->critical_supporting_reads;
}

/* the reference's value arrays and contig table, wrapped without a copy (every block is loaded
 * before the first voting run, core.c:3553-3558): the event stage and iteration two read them */
static svg_genome_arrays *svg_gen;

static int svg_gen_setup(global_context_t *gc)
{
	if (svg_gen) return 0;
	svg_value_block blk[100];
	int nb = gc->index_block_number, b;
	if (nb < 1 || nb > 100) return SVG_E_ARG;
	for (b = 0; b < nb; b++) {
		gene_value_index_t *v = &gc->all_value_indexes[b];
		blk[b].values = v->values;
		blk[b].start_point = v->start_point;
		blk[b].length = v->length;
		blk[b].start_base_offset = v->start_base_offset;
		blk[b].values_bytes = v->values_bytes;
	}
	gene_offset_t *ct = &gc->chromosome_table;
	return svg_genome_arrays_wrap(blk, nb, ct->read_offsets, ct->read_names, MAX_CHROMOSOME_NAME_LEN, (uint32_t)ct->total_offsets,
	                              ct->padding, 1, &svg_gen);
}

/* svg_ev_why: why the library cannot run this chunk's event stage (NULL: it can); decided once per
 * run by thread 0 (vote_stage) so that every thread takes the same path */

static const char *svg_events_unsupported(global_context_t *gc)
{
	const char *env = getenv("SVG_REF_EVENTSTAGE");
	if (env && env[0] == '1') return "SVG_REF_EVENTSTAGE=1";
	if (gc->config.space_type != GENE_SPACE_BASE) return "colour space";
	if (gc->config.do_fusion_detection || gc->config.do_long_del_detection) return "fusion / long-deletion detection";
	if (!gc->config.use_dynamic_programming_indel || gc->config.extending_search_indels) return "indel search other than dynamic programming";
	if (gc->config.multi_best_reads > 3) return "more than 3 records per read end";
	/* (svg_event keeps 40 inserted bases; an insertion is at most -I long) */
	if (gc->config.max_indel_length > 40) return "insertions may exceed 40 bases (-I > 40)";
	if (svg_gen_setup(gc)) return "the genome arrays could not be wrapped";
	return NULL;
}

/* the event table this run's thread adds to: its own (the reference's threads each fill one,
 * merged by finalise_indel_and_junction_thread, core.c:3452) or, with one thread, the global one */
typedef struct { HashTable *tab; unsigned int *total; } run_table;

static run_table run_table_of(global_context_t *gc, thread_context_t *tc)
{
	indel_context_t *ic = (indel_context_t *)gc->module_contexts[MODULE_INDEL_ID];
	indel_thread_context_t *itc = tc ? (indel_thread_context_t *)tc->module_thread_contexts[MODULE_INDEL_ID] : NULL;
	run_table T = {itc ? itc->event_entry_table : ic->event_entry_table, itc ? &itc->total_events : &ic->total_events};
	return T;
}

static chromosome_event_t *run_space(global_context_t *gc, thread_context_t *tc)
{
	indel_context_t *ic = (indel_context_t *)gc->module_contexts[MODULE_INDEL_ID];
	indel_thread_context_t *itc = tc ? (indel_thread_context_t *)tc->module_thread_contexts[MODULE_INDEL_ID] : NULL;
	return itc ? itc->event_space_dynamic : ic->event_space_dynamic;
}

/* the run's table as the library's: its events and every id list of its entry table, as they are */
static int table_in(global_context_t *gc, thread_context_t *tc, svg_events **out)
{
	run_table T = run_table_of(gc, tc);
	const chromosome_event_t *space = run_space(gc, tc);
	const int64_t n = *T.total, ns = T.tab->numOfElements;
	svg_event *ev = calloc((size_t)(n ? n : 1), sizeof(svg_event));
	uint32_t *pos = malloc(sizeof(uint32_t) * (size_t)(ns ? ns : 1)), *ids = calloc((size_t)(ns ? ns : 1) * 9, sizeof(uint32_t));
	uint8_t *cap = malloc((size_t)(ns ? ns : 1));
	int rc = ev && pos && ids && cap ? 0 : SVG_E_NOMEM;
	int64_t i, k = 0;
	for (i = 0; !rc && i < n; i++) event_to_svg(space + i, &ev[i]);
	for (i = 0; !rc && i < T.tab->numOfBuckets; i++)
		for (KeyValuePair *kv = T.tab->bucketArray[i]; kv && !rc; kv = kv->next) {
			const unsigned int *L = kv->value;
			const unsigned int c = L[0] & 0x0fffffff;
			if (k >= ns || c < 1 || c > 9) { rc = SVG_E_ARG; break; }
			pos[k] = (uint32_t)(uintptr_t)kv->key;
			cap[k] = (uint8_t)c;
			for (unsigned int j = 0; j < c; j++) {
				ids[k * 9 + j] = L[1 + j];
				if (!L[1 + j]) break;
			}
			k++;
		}
	svg_events *t = NULL;
	if (!rc) rc = svg_events_create(&t);
	if (!rc) rc = svg_events_load_sites(t, ev, n, pos, ids, cap, k);
	if (rc && t) { svg_events_destroy(t); t = NULL; }
	free(ev); free(pos); free(ids); free(cap);
	*out = t;
	return rc;
}

/* the library's table back into the run's: the events it had get their (updated) fields, the
 * new ones are added in order as local_add_indel_event / put_new_event add them
 * (core-indel.c:1498-1569, 1385-1419) -- the library put them into the same id lists the same way */
static int table_out(global_context_t *gc, thread_context_t *tc, const svg_events *t, int64_t n0)
{
	run_table T = run_table_of(gc, tc);
	const int64_t n = svg_events_count(t);
	svg_event *ev = malloc(sizeof(svg_event) * (size_t)(n ? n : 1));
	if (!ev) return SVG_E_NOMEM;
	int rc = svg_events_get(t, ev);
	/* (checked before anything is written: a failure leaves the run's table as it was) */
	for (int64_t i = n0; !rc && i < n; i++)
		if (ev[i].event_type == CHRO_EVENT_TYPE_INDEL && ev[i].indel_length < 0 && -ev[i].indel_length > ev[i].inserted_len) rc = SVG_E_ARG;
	chromosome_event_t *space = run_space(gc, tc);
	for (int64_t i = 0; !rc && i < n0; i++) event_to_ref(&ev[i], space + i);
	for (int64_t i = n0; !rc && i < n; i++) {
		const int no = (int)(*T.total)++;
		space = reallocate_event_space(gc, tc, no);
		chromosome_event_t *e = space + no;
		memset(e, 0, sizeof *e);
		event_to_ref(&ev[i], e);
		if (e->event_type == CHRO_EVENT_TYPE_INDEL && e->indel_length < 0) {
			char ins[MAX_INSERTION_LENGTH + 1];
			const int L = -e->indel_length;
			memcpy(ins, ev[i].inserted_bases, (size_t)L);
			ins[L] = 0;
			set_insertion_sequence(gc, tc, &e->inserted_bases, ins, L);
		}
		put_new_event(T.tab, e, no);
	}
	free(ev);
	return rc;
}

/* the library's event stage for reads [r0, r1) of the chunk: this block's fragile windows of those
 * reads and, in the final run, their tails (include/subread_events.h); NULL, or why it did not run
 * (the run's table is then as it was) */
static const char *tail_stage_lib(global_context_t *gc, thread_context_t *tc, uint64_t r0, uint64_t r1)
{
	static __thread char why[300];
	const svg_chunk_reads *c = &svg_chunk;
	const int ends = 1 + gc->input_reads.is_paired_end_reads, final = gc->is_final_voting_run;
	svg_params p;
	svg_fill_params(gc, &p);
	svg_event_params ep;
	svg_event_params_default(&ep);
	ep.dp_penalty_create_gap = gc->config.DP_penalty_create_gap;
	ep.dp_penalty_extend_gap = gc->config.DP_penalty_extend_gap;
	ep.dp_match_score = gc->config.DP_match_score;
	ep.dp_mismatch_penalty = gc->config.DP_mismatch_penalty;
	ep.report_multi_mapping_reads = gc->config.report_multi_mapping_reads;
	ep.quality_base = gc->config.phred_score_format == FASTQ_PHRED64 ? 'B' : '#';   /* read_quality_score, gene-algorithms.c:138 */
	ep.maximise_sensitivity_indel = gc->config.maximise_sensitivity_indel;
	svg_reads R[2], Q[2];
	const int ftype = gc->input_reads.first_read_file.file_type, quals = ftype != GENE_INPUT_FASTA && ftype != GENE_INPUT_GZIP_FASTA;
	for (int e = 0; e < ends; e++) {
		R[e] = (svg_reads){c->text[e], c->off[e] + r0, c->len[e] + r0, r1 - r0};
		Q[e] = (svg_reads){c->qual[e], c->off[e] + r0, c->len[e] + r0, r1 - r0};
	}
	/* this block's windows of these reads, numbered from r0 */
	svg_fragile_result fr = {0, svg_frag.n_slots, NULL, svg_frag.slots};
	const uint64_t w0 = svg_win[r0], w1 = svg_win[r1];
	if (w1 > w0) {
		fr.windows = malloc(sizeof(svg_fragile_window) * (size_t)(w1 - w0));
		if (!fr.windows) return "out of memory";
		memcpy(fr.windows, svg_frag.windows + w0, sizeof(svg_fragile_window) * (size_t)(w1 - w0));
		for (uint64_t w = 0; w < w1 - w0; w++) fr.windows[w].read -= (uint32_t)r0;
		fr.n_windows = w1 - w0;
	}
	if (!final && !fr.n_windows) return NULL;   /* nothing this run adds for these reads */
	svg_events *t = NULL;
	int rc = table_in(gc, tc, &t);
	const int64_t n0 = rc ? 0 : svg_events_count(t);
	if (!rc && !final)
		rc = svg_events_add_windows(t, svg_gen, &p, &ep, &R[0], ends == 2 ? &R[1] : NULL, &fr, gc->current_index_block_number);
	else if (!rc) {
		const uint64_t per = (uint64_t)ends * (uint64_t)gc->config.multi_best_reads;
		svg_mapping_result *out = (svg_mapping_result *)_global_retrieve_alignment_ptr(gc, 0, 0, 0) + r0 * per;
		const svg_subjunc_result *jout = p.do_breakpoint_detection ? (const svg_subjunc_result *)_global_retrieve_subjunc_ptr(gc, 0, 0, 0) + r0 * per : NULL;
		const uint16_t *bm = svg_bm ? svg_bm + r0 * (uint64_t)ends * SVG_BIG_MARGIN_WORDS : NULL;
		rc = svg_events_add_batch2(t, svg_gen, &p, &ep, &R[0], ends == 2 ? &R[1] : NULL, quals ? &Q[0] : NULL,
		                           ends == 2 && quals ? &Q[1] : NULL, r0, out, jout, bm, p.do_breakpoint_detection ? &fr : NULL);
	}
	if (!rc) rc = table_out(gc, tc, t, n0);
	if (rc) snprintf(why, sizeof why, "library event stage failed (%d): %s", rc, svg_last_error());
	svg_events_destroy(t);
	free(fr.windows);
	return rc ? why : NULL;
}

/* do_voting's per-read host work for reads [r0, r1) of the chunk: the library's, or the reference's
 * functions where it does not run */
static void tail_stage(global_context_t *gc, thread_context_t *tc, uint64_t r0, uint64_t r1)
{
	const char *why = svg_ev_why;
	if (!why) why = tail_stage_lib(gc, tc, r0, r1);
	svg_stage(ST_EVENTS, why);
	if (why) tail_stage_ref(gc, tc, r0, r1);
}

static void run_end(global_context_t *gc)
{
	chunk_free(&svg_chunk);
	memset(&svg_chunk, 0, sizeof svg_chunk);
	free(svg_win);
	svg_win = NULL;
	if (gc->is_final_voting_run) {
		svg_fragile_free(&svg_frag);
		free(svg_bm);
		svg_bm = NULL;
	}
}

/* one thread: the whole run */
int do_voting_gpu(global_context_t *gc, thread_context_t *tc)
{
	int rc = vote_stage(gc, tc);
	const double t0 = miltime();
	if (!rc) tail_stage(gc, tc, 0, svg_chunk.n);
	svg_t_tail += miltime() - t0;
	run_end(gc);
	svg_t_mark = miltime();
	return rc ? 1 : 0;
}

/* every one of the run's `nthreads` threads (run_in_thread, one do_voting each): thread 0 reads
 * and votes the chunk, then each thread does the per-read host work of a contiguous slice of it
 * into its own event tables, as the reference's threads do for the reads they fetch */
static pthread_barrier_t svg_bar;
static int svg_bar_n;
static volatile int svg_run_rc;

int do_voting_gpu_mt(global_context_t *gc, thread_context_t *tc, int nthreads)
{
	pthread_mutex_lock(&svg_sam_mu_init);
	if (svg_bar_n != nthreads) {
		if (svg_bar_n) pthread_barrier_destroy(&svg_bar);
		pthread_barrier_init(&svg_bar, NULL, (unsigned)nthreads);
		svg_bar_n = nthreads;
	}
	pthread_mutex_unlock(&svg_sam_mu_init);
	const int tid = tc->thread_id;
	if (tid == 0) svg_run_rc = vote_stage(gc, tc);
	pthread_barrier_wait(&svg_bar);
	const double t0 = miltime();
	if (!svg_run_rc) {
		const uint64_t n = svg_chunk.n;
		tail_stage(gc, tc, n * (uint64_t)tid / (uint64_t)nthreads, n * (uint64_t)(tid + 1) / (uint64_t)nthreads);
	}
	pthread_barrier_wait(&svg_bar);
	if (tid == 0) svg_t_tail += miltime() - t0;
	const int rc = svg_run_rc;
	if (tid == 0) run_end(gc);
	if (tid == 0) svg_t_mark = miltime();
	return rc ? 1 : 0;
}

/*
 * SAM emission of iteration two (include/subread_sam.h).  write_single_fragment (core.c:1888-2178)
 * hands each fragment's finished fields to add_buffered_fragment (core.c:1835-1884), which with
 * SAM output spins every -T thread on the output lock until the fragments before its own are out.
 * add_buffered_fragment_svg formats the same line(s) (svg_sam_format) and puts them in the
 * library's ordered sink, which writes them in the same order without any thread waiting.  BAM
 * output keeps the reference's own writer calls (SamBam_writer_add_read), which order themselves.
 */
#include "sambam-file.h"
#include "subread_sam.h"

static svg_sam_writer *svg_sam;
static SamBam_Writer *svg_bam_w;       /* the BAM writer whose file svg_sam writes (BAM output) */
static pthread_mutex_t svg_sam_mu = PTHREAD_MUTEX_INITIALIZER;

void add_buffered_fragment_svg(global_context_t *gc, thread_context_t *tc, subread_read_number_t pair_number,
	char *read_name1, unsigned int flags1, char *chro_name1, unsigned int chro_position1, int mapping_quality1, char *cigar1,
	char *next_chro_name1, unsigned int next_chro_pos1, int temp_len1, int read_len1,
	char *read_text1, char *qual_text1, char *additional_columns1,
	char *read_name2, unsigned int flags2, char *chro_name2, unsigned int chro_position2, int mapping_quality2, char *cigar2,
	char *next_chro_name2, unsigned int next_chro_pos2, int temp_len2, int read_len2,
	char *read_text2, char *qual_text2, char *additional_columns2,
	int all_locations, int this_location)
{
	const int pe = gc->input_reads.is_paired_end_reads;
	if (gc->config.is_BAM_output && !gc->config.is_input_read_order_required) {
		/* the reference's unordered per-thread BAM path (core.c:1849-1853) */
		SamBam_writer_add_read(gc->output_bam_writer, tc->thread_id, read_name1, flags1, chro_name1, chro_position1,
		                       mapping_quality1, cigar1, next_chro_name1, next_chro_pos1, temp_len1, read_len1, read_text1,
		                       qual_text1, additional_columns1, !pe);
		if (pe)
			SamBam_writer_add_read(gc->output_bam_writer, tc->thread_id, read_name2, flags2, chro_name2, chro_position2,
			                       mapping_quality2, cigar2, next_chro_name2, next_chro_pos2, temp_len2, read_len2,
			                       read_text2, qual_text2, additional_columns2, 1);
		return;
	}
	if (gc->config.is_BAM_output) {
		/* --keepReadOrder with BAM output: the reference's ordered path (core.c:1855-1881) -- wait
		 * for the fragments before this one, then write through the ordered writer (-1 / -2) */
		for (;;) {
			int fin = 0;
			subread_lock_occupy(&gc->output_lock);
			if (gc->last_written_fragment_number == pair_number - 1) {
				SamBam_writer_add_read(gc->output_bam_writer, -1, read_name1, flags1, chro_name1, chro_position1, mapping_quality1,
				                       cigar1, next_chro_name1, next_chro_pos1, temp_len1, read_len1, read_text1, qual_text1,
				                       additional_columns1, !pe);
				if (pe)
					SamBam_writer_add_read(gc->output_bam_writer, -2, read_name2, flags2, chro_name2, chro_position2, mapping_quality2,
					                       cigar2, next_chro_name2, next_chro_pos2, temp_len2, read_len2, read_text2, qual_text2,
					                       additional_columns2, 1);
				if (all_locations <= this_location + 1) gc->last_written_fragment_number = pair_number;
				fin = 1;
			}
			subread_lock_release(&gc->output_lock);
			if (fin) return;
			usleep(2);
		}
	}
	pthread_mutex_lock(&svg_sam_mu);
	if (!svg_sam && svg_sam_writer_open(gc->output_sam_fp, &svg_sam))
		SUBREADprintf("svg_sam_writer_open: %s\n", svg_last_error());
	/* run_maybe_threads sets last_written_fragment_number = -1 before every iteration two
	 * (core.c:3384-3386), which this function otherwise leaves alone: a new chunk */
	if (svg_sam && gc->last_written_fragment_number == -1) {
		if (svg_sam_writer_begin_chunk(svg_sam, gc->processed_reads_in_chunk)) {
			/* fragments of the last chunk never completed (a fragment that was never put): the
			 * reference's error path for a short output (output_sam_is_full) rather than a
			 * silently truncated SAM */
			SUBREADprintf("svg_sam_writer_begin_chunk: %s\n", svg_last_error());
			gc->output_sam_is_full = 1;
		}
		gc->last_written_fragment_number = -2;
	}
	pthread_mutex_unlock(&svg_sam_mu);
	if (!svg_sam) { gc->output_sam_is_full = 1; return; }
	svg_sam_record r1 = {read_name1, (int32_t)flags1, chro_name1, chro_position1, mapping_quality1, cigar1, next_chro_name1,
	                     next_chro_pos1, temp_len1, read_text1, qual_text1, additional_columns1};
	svg_sam_record r2 = {read_name2, (int32_t)flags2, chro_name2, chro_position2, mapping_quality2, cigar2, next_chro_name2,
	                     next_chro_pos2, temp_len2, read_text2, qual_text2, additional_columns2};
	size_t cap = 4096 + 2 * (size_t)(read_len1 + read_len2) + strlen(additional_columns1) +
	             (pe ? strlen(additional_columns2) : 0) + strlen(read_name1) + (pe ? strlen(read_name2) : 0) +
	             strlen(cigar1) + (pe ? strlen(cigar2) : 0) + strlen(qual_text1) + (pe ? strlen(qual_text2) : 0);
	char stackbuf[8192], *buf = cap <= sizeof stackbuf ? stackbuf : malloc(cap);
	int64_t n1 = buf ? svg_sam_format(&r1, buf, cap) : -1, n2 = 0;
	if (n1 >= 0 && pe) n2 = svg_sam_format(&r2, buf + n1, cap - (size_t)n1);
	if (n1 < 0 || n2 < 0) {
		SUBREADprintf("svg_sam_format: record of fragment %lld does not fit\n", (long long)pair_number);
		gc->output_sam_is_full = 1;
	} else {
		/* the reference's fragment is complete once all_locations <= this_location + 1
		 * (core.c:1875): an unmapped fragment comes with all_locations = 0 */
		const int all = all_locations > this_location + 1 ? all_locations : this_location + 1;
		int rc = svg_sam_writer_put(svg_sam, pair_number, this_location, all, buf, (size_t)(n1 + n2));
		if (rc || svg_sam_writer_failed(svg_sam)) {
			SUBREADprintf("svg_sam_writer_put (fragment %lld, location %d of %d): error %d, write %s\n", (long long)pair_number,
			              this_location, all_locations, rc, svg_sam_writer_failed(svg_sam) ? "failed" : "ok");
			gc->output_sam_is_full = 1;
		}
	}
	if (buf != stackbuf) free(buf);
}

/* the sink is flushed at each chunk's last fragment; closed (and its FILE* flushed) once the
 * run is over -- the harness calls this from its end-of-run hook */
int svg_sam_finish(void)
{
	int rc = 0;
	/* a fragment never put (or a short write) fails the run as the reference's output_sam_is_full
	 * does (destroy_global_context, core.c:4270-4275: no output file, exit status 1) */
	const int bam = svg_sam && svg_sam_writer_is_bam(svg_sam);
	if (svg_sam && (rc = svg_sam_writer_close(svg_sam))) SUBREADprintf("svg_sam_writer_close: %s\n", svg_last_error());
	svg_sam = NULL;
	/* (the BAM writer closes the file after this: its end-of-file block follows our last block) */
	if (bam && svg_bam_w) svg_bam_w->current_BAM_pos = ftello(svg_bam_w->bam_fp);
	svg_stages_print(stderr);
	if (getenv("SVG_REF_TIMING"))
		fprintf(stderr, "SVG_DROPIN_VOTING index_open=%.6f read_chunk=%.6f vote_call=%.6f fragile=%.6f tail=%.6f to_anti=%.6f "
		        "anti=%.6f to_it2=%.6f realign=%.6f\n",
		        svg_t_open, svg_t_read, svg_t_vote, svg_t_frag, svg_t_tail, svg_t_to_anti, svg_t_anti, svg_t_to_it2, svg_t_realign);
	return rc;
}

/*
 * The reads of a chunk, parsed once (drop-in build).  The reference parses every read of a chunk
 * in every pass over it -- the voting run of each index block and iteration two -- one read at a
 * time under the input lock (fetch_next_read_pair, core.c:1121-1211), so with the vote on the GPU
 * the serial parse is what iteration two waits on.  fetch_next_read_pair_svg is that function
 * (same parser calls, same trimming, secondary-read skip, read numbering and -S reversal) with a
 * cache: the first pass over a chunk parses and keeps each read as it hands it out; a later pass
 * over the same chunk (the reference rewinds to the chunk start it saved,
 * current_circle_start_position_file1, core.c:3487-3490,3523-3529) is served from the cache in the
 * same order, and the input file is left where the rewind put it -- the reference seeks to the
 * saved chunk end itself afterwards (go_chunk_nextchunk, core.c:3531-3537).  Colour space is never
 * cached.
 */
#include "input-files.h"
#include "gene-algorithms.h"

typedef struct {
	char *buf;                         /* name\0 text\0 qual\0 per read end, back to back */
	uint64_t len, cap;
	uint64_t *at;                      /* read r, end e: offset at[r * 2 + e] */
	int *rl;                           /* read lengths, [r * 2 + e] */
	uint64_t n, ncap;
	int complete;                      /* the parse pass reached the chunk's end */
	gene_inputfile_position_t start1;  /* the chunk's start (current_circle_start_position_file1) */
} svg_read_cache;

static svg_read_cache svg_rc;
static int svg_pass_cached;            /* the current pass is served from svg_rc */

static int rc_put(int e, const char *name, const char *text, const char *qual, int rl)
{
	const size_t nn = strlen(name) + 1, tn = (size_t)rl + 1, qn = qual ? strlen(qual) + 1 : 1;
	if (svg_rc.len + nn + tn + qn > svg_rc.cap) {
		uint64_t nc = (svg_rc.cap + nn + tn + qn) * 2 + (1 << 20);
		char *nb = realloc(svg_rc.buf, nc);
		if (!nb) return -1;
		svg_rc.buf = nb;
		svg_rc.cap = nc;
	}
	svg_rc.at[svg_rc.n * 2 + e] = svg_rc.len;
	svg_rc.rl[svg_rc.n * 2 + e] = rl;
	memcpy(svg_rc.buf + svg_rc.len, name, nn); svg_rc.len += nn;
	memcpy(svg_rc.buf + svg_rc.len, text, tn); svg_rc.len += tn;
	if (qual) memcpy(svg_rc.buf + svg_rc.len, qual, qn); else svg_rc.buf[svg_rc.len] = 0;
	svg_rc.len += qn;
	return 0;
}

static void rc_get(uint64_t r, int e, char *name, char *text, char *qual, int *rl)
{
	const char *p = svg_rc.buf + svg_rc.at[r * 2 + e];
	const size_t nn = strlen(p) + 1;
	strcpy(name, p);
	*rl = svg_rc.rl[r * 2 + e];
	memcpy(text, p + nn, (size_t)*rl + 1);
	if (qual) strcpy(qual, p + nn + *rl + 1);
}

/*
 * geinput_next_read_trim's plain-FASTQ branch (input-files.c:982-1093, with read_line_noempty
 * :209-261 and SKIP_LINE :650) restated with the FILE's lock taken once per read (flockfile +
 * getc_unlocked) instead of once per character (fgetc through geinput_getc, :197): the same bytes
 * consumed, the same name / text / quality strings and return values, the file position where the
 * reference's parse leaves it (chunk rewinds and saved positions see no difference).  Other input
 * types take the reference's own function.
 */
int trim_read_inner(char *read_text, char *qual_text, int rlen, short t_5, short t_3);
srInt_64 tell_current_line_no(gene_input_t *input);

static int fq_line_noempty(FILE *fp, int max_len, char *buff)
{
	int ret = 0;
	for (;;) {
		const char ch = (char)getc_unlocked(fp);
		if (ch == EOF) break;
		if (ch == '\n') {
			if (ret) break;
		} else if (ret < max_len - 1) buff[ret++] = ch;
	}
	buff[ret] = 0;
	return ret;
}

/*
 * Bulk reading of plain FASTQ while the binding's own chunk read runs (read_chunk): the parse
 * below takes its bytes from a 4 MB buffer filled by fread and finds line ends with memchr instead
 * of one getc per character; at the end of the chunk read the FILE is put back (fseeko) exactly
 * where the character-wise parse would have left it -- nothing else touches the FILE in between
 * (preloading is a no-op for plain files, input-files.c:199-203), and the reference's own
 * position bookkeeping (geinput_tell = ftello, :684-698) only runs outside.  A byte 0xFF ends a
 * line or the input as the reference's `char` comparisons with EOF make it do.
 */
typedef struct {
	FILE *fp;
	char *buf;
	size_t cap, lo, hi;               /* unread bytes buf[lo..hi) */
	off_t pos;                        /* file offset of buf[hi] */
	int on, eof;
} svg_fqbuf;
static svg_fqbuf svg_fqb[2];

static void fqb_begin(gene_input_t *ginp1, gene_input_t *ginp2)
{
	gene_input_t *in[2] = {ginp1, ginp2};
	for (int e = 0; e < 2; e++) {
		svg_fqbuf *b = &svg_fqb[e];
		b->on = 0;
		if (!in[e] || in[e]->file_type != GENE_INPUT_FASTQ) continue;
		if (!b->buf) {
			b->cap = (size_t)4 << 20;
			if (!(b->buf = malloc(b->cap))) continue;
		}
		b->fp = (FILE *)in[e]->input_fp;
		b->pos = ftello(b->fp);
		if (b->pos < 0) continue;
		b->lo = b->hi = 0;
		b->eof = 0;
		b->on = 1;
	}
}

static void fqb_end(void)
{
	for (int e = 0; e < 2; e++) {
		svg_fqbuf *b = &svg_fqb[e];
		if (!b->on) continue;
		fseeko(b->fp, b->pos - (off_t)(b->hi - b->lo), SEEK_SET);
		b->on = 0;
	}
}

static svg_fqbuf *fqb_of(FILE *fp)
{
	for (int e = 0; e < 2; e++)
		if (svg_fqb[e].on && svg_fqb[e].fp == fp) return &svg_fqb[e];
	return NULL;
}

/* more bytes: 0 at the end of the file */
static size_t fqb_fill(svg_fqbuf *b)
{
	if (b->lo == b->hi) b->lo = b->hi = 0;
	else if (b->lo > 0) {
		memmove(b->buf, b->buf + b->lo, b->hi - b->lo);
		b->hi -= b->lo;
		b->lo = 0;
	}
	if (b->eof || b->hi == b->cap) return b->hi - b->lo;
	const size_t got = fread(b->buf + b->hi, 1, b->cap - b->hi, b->fp);
	if (got == 0) b->eof = 1;
	b->hi += got;
	b->pos += (off_t)got;
	return got;
}

/* getc_unlocked as a signed char (EOF = -1, and so is byte 0xFF) */
static inline int fqb_getc(svg_fqbuf *b)
{
	if (b->lo == b->hi && fqb_fill(b) == 0) return -1;
	return (signed char)b->buf[b->lo++];
}

/* fq_line_noempty from the buffer: leading newlines skipped, the line copied up to max_len - 1
 * characters (the rest consumed), ended by '\n' (consumed), 0xFF (consumed) or the end of file */
static int fqb_line_noempty(svg_fqbuf *b, int max_len, char *buff)
{
	int ret = 0;
	for (;;) {
		if (b->lo == b->hi && fqb_fill(b) == 0) break;
		const char *p = b->buf + b->lo;
		size_t n = b->hi - b->lo;
		if (ret == 0) {
			size_t k = 0;
			while (k < n && p[k] == '\n') k++;
			b->lo += k;
			if (k == n) continue;
			p += k;
			n -= k;
		}
		const char *nl = memchr(p, '\n', n);
		size_t take = nl ? (size_t)(nl - p) : n;
		const char *ff = memchr(p, 0xff, take);
		if (ff) take = (size_t)(ff - p);
		const size_t room = ret < max_len - 1 ? (size_t)(max_len - 1 - ret) : 0;
		const size_t cp = take < room ? take : room;
		memcpy(buff + ret, p, cp);
		ret += (int)cp;
		b->lo += take;
		if (ff || nl) { b->lo++; break; }   /* the terminating '\n' or 0xFF byte is consumed */
	}
	buff[ret] = 0;
	return ret;
}

static int fq_next_read_bulk(svg_fqbuf *b, gene_input_t *input, char *read_name, char *read_string, char *quality_string,
                             short trim_5, short trim_3)
{
	int nch, ret;
	do nch = fqb_getc(b); while (nch == '\n');
	if (nch == -1) return -1;
	if (nch != '@') {
		fseeko(b->fp, b->pos - (off_t)(b->hi - b->lo), SEEK_SET);   /* the message counts lines up to here */
		SUBREADprintf("ERROR: a format issue %d is found on the %lld-th line in input file '%s'.\nProgram aborted.\n", nch,
		              (long long)tell_current_line_no(input), input->filename);
		return -1;
	}
	fqb_line_noempty(b, MAX_READ_NAME_LEN, read_name);
	for (int cursor = 1; read_name[cursor]; cursor++)
		if (read_name[cursor] == ' ' || read_name[cursor] == '\t') { read_name[cursor] = 0; break; }
	ret = fqb_line_noempty(b, MAX_READ_LENGTH, read_string);
	do nch = fqb_getc(b); while (nch == '\n');
	if (nch != '+') {
		fseeko(b->fp, b->pos - (off_t)(b->hi - b->lo), SEEK_SET);
		SUBREADprintf("ERROR: a format issue %c is found on the %lld-th line in input file '%s'.\nProgram aborted.\n", nch,
		              (long long)tell_current_line_no(input), input->filename);
		return -1;
	}
	nch = ' ';
	while (nch != -1 && nch != '\n') nch = fqb_getc(b);
	if (quality_string) fqb_line_noempty(b, MAX_READ_LENGTH, quality_string);
	else {
		int content = 0;
		nch = ' ';
		while (nch != -1 && (nch != '\n' || !content)) { nch = fqb_getc(b); content += nch != '\n'; }
	}
	if (trim_5 || trim_3) ret = trim_read_inner(read_string, quality_string, ret, trim_5, trim_3);
	return ret;
}

static int fq_next_read(gene_input_t *input, char *read_name, char *read_string, char *quality_string, short trim_5,
                        short trim_3)
{
	FILE *fp = (FILE *)input->input_fp;
	svg_fqbuf *bq = fqb_of(fp);
	if (bq) return fq_next_read_bulk(bq, input, read_name, read_string, quality_string, trim_5, trim_3);
	signed char nch;
	int ret;
	flockfile(fp);
	do nch = (signed char)getc_unlocked(fp); while (nch == '\n');
	if (nch == EOF) { funlockfile(fp); return -1; }
	if (nch != '@') {
		funlockfile(fp);
		SUBREADprintf("ERROR: a format issue %d is found on the %lld-th line in input file '%s'.\nProgram aborted.\n", nch,
		              (long long)tell_current_line_no(input), input->filename);
		return -1;
	}
	fq_line_noempty(fp, MAX_READ_NAME_LEN, read_name);
	for (int cursor = 1; read_name[cursor]; cursor++)
		if (read_name[cursor] == ' ' || read_name[cursor] == '\t') { read_name[cursor] = 0; break; }
	ret = fq_line_noempty(fp, MAX_READ_LENGTH, read_string);
	do nch = (signed char)getc_unlocked(fp); while (nch == '\n');
	if (nch != '+') {
		funlockfile(fp);
		SUBREADprintf("ERROR: a format issue %c is found on the %lld-th line in input file '%s'.\nProgram aborted.\n", nch,
		              (long long)tell_current_line_no(input), input->filename);
		return -1;
	}
	nch = ' ';
	while (nch != EOF && nch != '\n') nch = (signed char)getc_unlocked(fp);
	if (quality_string) fq_line_noempty(fp, MAX_READ_LENGTH, quality_string);
	else {
		int content = 0;
		nch = ' ';
		while (nch != EOF && (nch != '\n' || !content)) { nch = (signed char)getc_unlocked(fp); content += nch != '\n'; }
	}
	funlockfile(fp);
	if (trim_5 || trim_3) ret = trim_read_inner(read_string, quality_string, ret, trim_5, trim_3);
	return ret;
}

static int next_read_trim(gene_input_t *input, char *read_name, char *read_string, char *quality_string, short trim_5,
                          short trim_3, int *is_secondary)
{
	if (input->file_type == GENE_INPUT_FASTQ && read_name)
		return fq_next_read(input, read_name, read_string, quality_string, trim_5, trim_3);
	return geinput_next_read_trim(input, read_name, read_string, quality_string, trim_5, trim_3, is_secondary);
}

int fetch_next_read_pair_svg(global_context_t *gc, thread_context_t *tc, gene_input_t *ginp1, gene_input_t *ginp2,
                             int *read_len_1, int *read_len_2, char *read_name_1, char *read_name_2, char *read_text_1,
                             char *read_text_2, char *qual_text_1, char *qual_text_2, int remove_color_head,
                             subread_read_number_t *read_no_in_chunk)
{
	(void)tc;
	int rl1 = 0, rl2 = 0, is_second_R1, is_second_R2;
	subread_read_number_t this_number = -1;
	const int cacheable = gc->config.space_type != GENE_SPACE_COLOR && gc->input_reads.first_read_file.file_type != GENE_INPUT_BCL;
	if (!svg_pass_cached) {
		geinput_preload_buffer(ginp1, &gc->input_reads.input_lock);
		if (ginp2) geinput_preload_buffer(ginp2, &gc->input_reads.input_lock);
	}
	subread_lock_occupy(&gc->input_reads.input_lock);
	if (gc->running_processed_reads_in_chunk == 0) {
		/* a pass begins: the same chunk as the complete cache -> serve it; else parse, refill */
		svg_pass_cached = cacheable && svg_rc.complete &&
		                  !memcmp(&svg_rc.start1, &gc->current_circle_start_position_file1, sizeof svg_rc.start1);
		if (!svg_pass_cached && cacheable) {
			svg_rc.n = svg_rc.len = 0;
			svg_rc.complete = 0;
			memcpy(&svg_rc.start1, &gc->current_circle_start_position_file1, sizeof svg_rc.start1);
		}
	}
	if (svg_pass_cached) {
		if (gc->running_processed_reads_in_chunk < (subread_read_number_t)svg_rc.n) {
			this_number = gc->running_processed_reads_in_chunk++;
			subread_lock_release(&gc->input_reads.input_lock);
			rc_get((uint64_t)this_number, 0, read_name_1, read_text_1, qual_text_1, read_len_1);
			if (ginp2) rc_get((uint64_t)this_number, 1, read_name_2, read_text_2, qual_text_2, read_len_2);
			*read_no_in_chunk = this_number;
			return 0;
		}
		subread_lock_release(&gc->input_reads.input_lock);
		*read_no_in_chunk = -1;
		return 1;
	}
	if (gc->running_processed_reads_in_chunk < gc->config.reads_per_chunk) {
		do {
			is_second_R1 = 0; is_second_R2 = 0;
			rl1 = next_read_trim(ginp1, read_name_1, read_text_1, qual_text_1, gc->config.read_trim_5,
			                     gc->config.read_trim_3, &is_second_R1);
			if (gc->config.space_type == GENE_SPACE_COLOR && remove_color_head && isalpha(read_text_1[0])) {
				int xk1;
				for (xk1 = 2; read_text_1[xk1]; xk1++) read_text_1[xk1 - 2] = read_text_1[xk1];
				read_text_1[xk1 - 2] = 0;
			}
			if (ginp2) {
				rl2 = next_read_trim(ginp2, read_name_2, read_text_2, qual_text_2, gc->config.read_trim_5,
				                     gc->config.read_trim_3, &is_second_R2);
				if (gc->config.space_type == GENE_SPACE_COLOR && remove_color_head && isalpha(read_text_2[0])) {
					int xk1;
					for (xk1 = 2; read_text_2[xk1]; xk1++) read_text_2[xk1 - 2] = read_text_2[xk1];
					read_text_2[xk1 - 2] = 0;
				}
			}
			if (rl1 <= 0 || (rl2 <= 0 && ginp2)) break;
		} while (is_second_R1 || is_second_R2);
		if (rl1 > 0 || (rl2 > 0 && ginp2)) this_number = gc->running_processed_reads_in_chunk++;
	}
	int ok = this_number >= 0 && rl1 > 0 && (rl2 > 0 || !ginp2);
	if (gc->config.space_type == GENE_SPACE_COLOR) { rl1 -= 1; rl2 -= 1; }
	if (ok && gc->config.space_type != GENE_SPACE_COLOR) {
		if (gc->config.is_first_read_reversed) {
			reverse_read(read_text_1, rl1, gc->config.space_type);
			if (qual_text_1) reverse_quality(qual_text_1, rl1);
		}
		if (ginp2 && gc->config.is_second_read_reversed) {
			reverse_read(read_text_2, rl2, gc->config.space_type);
			if (qual_text_2) reverse_quality(qual_text_2, rl2);
		}
		/* keep the read as handed out (the cache is filled in read-number order under the lock) */
		if (cacheable && (uint64_t)this_number == svg_rc.n) {
			if (svg_rc.n == svg_rc.ncap) {
				svg_rc.ncap = svg_rc.ncap ? 2 * svg_rc.ncap : 1 << 16;
				svg_rc.at = realloc(svg_rc.at, svg_rc.ncap * 2 * sizeof(uint64_t));
				svg_rc.rl = realloc(svg_rc.rl, svg_rc.ncap * 2 * sizeof(int));
			}
			if (!svg_rc.at || !svg_rc.rl || rc_put(0, read_name_1, read_text_1, qual_text_1, rl1) ||
			    (ginp2 && rc_put(1, read_name_2, read_text_2, qual_text_2, rl2)))
				svg_rc.complete = -1;   /* out of memory: never served */
			else svg_rc.n++;
		}
	} else if (this_number < 0 && cacheable && svg_rc.complete == 0) svg_rc.complete = 1;   /* the pass ended */
	subread_lock_release(&gc->input_reads.input_lock);
	if (ginp2 && rl1 * rl2 <= 0 && (rl1 > 0 || rl2 > 0)) {
		if (!gc->input_reads.is_internal_error) SUBREADprintf("\nERROR: two input files have different amounts of reads.\n\n");
		gc->input_reads.is_internal_error = 1;
		*read_no_in_chunk = -1;
		return 1;
	} else if (rl1 > 0 && (rl2 > 0 || !ginp2) && this_number >= 0) {
		if (gc->config.space_type == GENE_SPACE_COLOR) {
			if (gc->config.is_first_read_reversed) {
				reverse_read(read_text_1, rl1, gc->config.space_type);
				if (qual_text_1) reverse_quality(qual_text_1, rl1);
			}
			if (ginp2 && gc->config.is_second_read_reversed) {
				reverse_read(read_text_2, rl2, gc->config.space_type);
				if (qual_text_2) reverse_quality(qual_text_2, rl2);
			}
		}
		*read_no_in_chunk = this_number;
		*read_len_1 = rl1;
		if (ginp2) *read_len_2 = rl2;
		return 0;
	}
	*read_no_in_chunk = -1;
	return 1;
}

#ifdef SVG_DROPIN_DO_VOTING
/*
 * Harness build (linked with -Wl,--wrap=gehash_load,... in oracle/Makefile).  The reference's CPU hash table (gehash_load, sorted-hashtable.c:1390; read_chunk_circles loads
 * one block at a time, core.c:3576) is what its own voting probes; with the vote on the GPU
 * (svg_index_open holds every block in HBM) nothing of the align / subjunc paths reads it.  The
 * drop-in therefore records the file and its index_gap (the one field the reference reads outside
 * the table's own functions, core.c:3088, core-junction.c:5172) and loads the table only if a
 * table function is ever called on it (long-indel reassembly, methylation mode).
 */
#include "sorted-hashtable.h"

#define SVG_LAZY_MAX 8
static struct { gehash_t *t; char fname[MAX_FILE_NAME_LENGTH + 40]; int loaded; } svg_lazy[SVG_LAZY_MAX];
static pthread_mutex_t svg_lazy_mu = PTHREAD_MUTEX_INITIALIZER;

int __real_gehash_load(gehash_t *the_table, const char fname[]);

static int tab_index_gap(const char *fname, int *gap, int *padding)
{
	FILE *fp = fopen(fname, "rb");
	char magic[8];
	if (!fp) return -1;
	int rc = -1;
	if (fread(magic, 1, 8, fp) == 8 && !memcmp(magic, "2subindx", 8))
		for (;;) {
			short k, l, v = 0;
			if (fread(&k, 2, 1, fp) != 1) break;
			if (!k) { rc = 0; break; }
			if (fread(&l, 2, 1, fp) != 1) break;
			if (l == 2 && fread(&v, 2, 1, fp) == 1) {
				if (k == 0x0101) *gap = v;
				else if (k == 0x0102) *padding = v;
			} else if (fseek(fp, l, SEEK_CUR)) break;
		}
	fclose(fp);
	return rc;
}

int __wrap_gehash_load(gehash_t *t, const char fname[])
{
	int gap = 0, padding = 0, i;
	if (tab_index_gap(fname, &gap, &padding) || gap < 1) return __real_gehash_load(t, fname);
	pthread_mutex_lock(&svg_lazy_mu);
	for (i = 0; i < SVG_LAZY_MAX && svg_lazy[i].t && svg_lazy[i].t != t; i++) ;
	if (i == SVG_LAZY_MAX) { pthread_mutex_unlock(&svg_lazy_mu); return __real_gehash_load(t, fname); }
	svg_lazy[i].t = t;
	snprintf(svg_lazy[i].fname, sizeof svg_lazy[i].fname, "%s", fname);
	svg_lazy[i].loaded = 0;
	pthread_mutex_unlock(&svg_lazy_mu);
	/* an empty table gehash_destory frees nothing from (core.c:3609) */
	memset(t->malloc_ptr, 0, sizeof(t->malloc_ptr));
	t->buckets = NULL;
	t->buckets_number = 0;
	t->current_items = 0;
	t->index_gap = gap;
	t->padding = padding;
	t->is_small_table = 0;
	t->free_item_only = 0;
	return 0;
}

static void lazy_ensure(gehash_t *t)
{
	pthread_mutex_lock(&svg_lazy_mu);
	for (int i = 0; i < SVG_LAZY_MAX; i++)
		if (svg_lazy[i].t == t && !svg_lazy[i].loaded) {
			svg_lazy[i].loaded = 1;
			if (__real_gehash_load(t, svg_lazy[i].fname)) SUBREADprintf("lazy gehash_load of %s failed\n", svg_lazy[i].fname);
		}
	pthread_mutex_unlock(&svg_lazy_mu);
}

size_t __real_gehash_go_q(gehash_t *the_table, gehash_key_t raw_key, int offset, int read_len, int is_reversed,
                          gene_vote_t *vote, int indel_tolerance, int subread_number, unsigned int low_border,
                          unsigned int high_border);
size_t __wrap_gehash_go_q(gehash_t *the_table, gehash_key_t raw_key, int offset, int read_len, int is_reversed,
                          gene_vote_t *vote, int indel_tolerance, int subread_number, unsigned int low_border,
                          unsigned int high_border)
{
	lazy_ensure(the_table);
	return __real_gehash_go_q(the_table, raw_key, offset, read_len, is_reversed, vote, indel_tolerance, subread_number,
	                          low_border, high_border);
}

size_t __real_gehash_go_X(gehash_t *the_table, gehash_key_t raw_key, int offset, int read_len, int is_reversed,
                          gene_vote_t *vote, int indel_tolerance, int subread_number, unsigned int low_border,
                          unsigned int high_border, int run_round, unsigned int *shift_indel_locs, unsigned int *shift_indel_NO);
size_t __wrap_gehash_go_X(gehash_t *the_table, gehash_key_t raw_key, int offset, int read_len, int is_reversed,
                          gene_vote_t *vote, int indel_tolerance, int subread_number, unsigned int low_border,
                          unsigned int high_border, int run_round, unsigned int *shift_indel_locs, unsigned int *shift_indel_NO)
{
	lazy_ensure(the_table);
	return __real_gehash_go_X(the_table, raw_key, offset, read_len, is_reversed, vote, indel_tolerance, subread_number,
	                          low_border, high_border, run_round, shift_indel_locs, shift_indel_NO);
}

size_t __real_gehash_go_q_CtoT(gehash_t *the_table, gehash_key_t key, int offset, int read_len, int is_reversed,
                               gene_vote_t *vote, gene_vote_number_t weight, int max_match_number, int indel_tolerance,
                               int subread_number, int max_error_bases, unsigned int low_border, unsigned int high_border);
size_t __wrap_gehash_go_q_CtoT(gehash_t *the_table, gehash_key_t key, int offset, int read_len, int is_reversed,
                               gene_vote_t *vote, gene_vote_number_t weight, int max_match_number, int indel_tolerance,
                               int subread_number, int max_error_bases, unsigned int low_border, unsigned int high_border)
{
	lazy_ensure(the_table);
	return __real_gehash_go_q_CtoT(the_table, key, offset, read_len, is_reversed, vote, weight, max_match_number,
	                               indel_tolerance, subread_number, max_error_bases, low_border, high_border);
}

size_t __real_gehash_go_q_tolerable(gehash_t *the_table, gehash_key_t key, int offset, int read_len, int is_reversed,
                                    gene_vote_t *vote, gene_vote_number_t weight, gene_quality_score_t quality,
                                    int max_match_number, int indel_tolerance, int subread_number, int max_error_bases,
                                    int subread_len, unsigned int low_border, unsigned int high_border);
size_t __wrap_gehash_go_q_tolerable(gehash_t *the_table, gehash_key_t key, int offset, int read_len, int is_reversed,
                                    gene_vote_t *vote, gene_vote_number_t weight, gene_quality_score_t quality,
                                    int max_match_number, int indel_tolerance, int subread_number, int max_error_bases,
                                    int subread_len, unsigned int low_border, unsigned int high_border)
{
	lazy_ensure(the_table);
	return __real_gehash_go_q_tolerable(the_table, key, offset, read_len, is_reversed, vote, weight, quality,
	                                    max_match_number, indel_tolerance, subread_number, max_error_bases, subread_len,
	                                    low_border, high_border);
}

/* harness build: core.o's fetch_next_read_pair is weak, every call site lands here */
int fetch_next_read_pair(global_context_t *gc, thread_context_t *tc, gene_input_t *ginp1, gene_input_t *ginp2,
                         int *read_len_1, int *read_len_2, char *read_name_1, char *read_name_2, char *read_text_1,
                         char *read_text_2, char *qual_text_1, char *qual_text_2, int remove_color_head,
                         subread_read_number_t *read_no_in_chunk)
{
	return fetch_next_read_pair_svg(gc, tc, ginp1, ginp2, read_len_1, read_len_2, read_name_1, read_name_2, read_text_1,
	                                read_text_2, qual_text_1, qual_text_2, remove_color_head, read_no_in_chunk);
}

/* harness build: the reference's core.o is compiled with add_buffered_fragment weak (below) */
void add_buffered_fragment(global_context_t *gc, thread_context_t *tc, subread_read_number_t pair_number,
	char *read_name1, unsigned int flags1, char *chro_name1, unsigned int chro_position1, int mapping_quality1, char *cigar1,
	char *next_chro_name1, unsigned int next_chro_pos1, int temp_len1, int read_len1,
	char *read_text1, char *qual_text1, char *additional_columns1,
	char *read_name2, unsigned int flags2, char *chro_name2, unsigned int chro_position2, int mapping_quality2, char *cigar2,
	char *next_chro_name2, unsigned int next_chro_pos2, int temp_len2, int read_len2,
	char *read_text2, char *qual_text2, char *additional_columns2,
	int all_locations, int this_location)
{
	add_buffered_fragment_svg(gc, tc, pair_number, read_name1, flags1, chro_name1, chro_position1, mapping_quality1, cigar1,
	                          next_chro_name1, next_chro_pos1, temp_len1, read_len1, read_text1, qual_text1,
	                          additional_columns1, read_name2, flags2, chro_name2, chro_position2, mapping_quality2, cigar2,
	                          next_chro_name2, next_chro_pos2, temp_len2, read_len2, read_text2, qual_text2,
	                          additional_columns2, all_locations, this_location);
}
#endif

#ifdef SVG_DROPIN_DO_VOTING
/*
 * Harness build only (oracle/Makefile `dropin`): the reference's core.o is compiled with
 * do_voting weak, so this definition takes run_in_thread's call (core.c:3366-3368).  Thread 0
 * (or the single -T 1 caller) reads the whole chunk and feeds it to the GPU, so read numbers
 * stay sequential; then every voting thread does the per-read host work of its slice of the
 * chunk (do_voting_gpu_mt).  The device is SVG_DEVICE (default 0).
 */

/*
 * Iteration two (harness build: core.o's do_iteration_two is weak; the reference's own stays
 * reachable as ref_do_iteration_two, an alias oracle/Makefile adds).  run_maybe_threads
 * (core.c:3379-3461) calls do_iteration_two from each of the run's -T threads after the chunk's
 * anti-supporting read scan and remove_neighbour (core.c:3629-3638); thread 0 (or the only
 * caller) runs the library's iteration two (include/subread_realign.h, svg_realign_chunk) over
 * the whole chunk with -T worker threads and the others return at once.  Inputs are the chunk's
 * reads as fetch_next_read_pair handed them out (the read cache above), the bigtable records,
 * the reference's merged event table, its value arrays and contig table; outputs go where the
 * reference's go: SAM lines to the ordered sink, final_counted_reads / junction flanking back
 * into the event table (add_realignment_event_support, core.c:2364-2379; the VCF / BED writers
 * read them), the counters into the thread context (core.c:3433-3444), the expected-TLEN state
 * into the global context.  Configurations the library does not cover (BAM output, colour space,
 * fusion / long-deletion detection, annotation exon scoring, scRNA input) and SVG_REF_ITER2=1
 * keep the reference's own iteration two.
 */
#include "subread_realign.h"

int ref_do_iteration_two(global_context_t *gc, thread_context_t *tc);
void print_in_box(int line_width, int is_boundary, int options, char *pattern, ...);

static svg_realign *svg_it2;

/* why iteration two of this chunk is the reference's (NULL: the library's) */
static const char *svg_it2_unsupported(global_context_t *gc)
{
	const char *e = getenv("SVG_REF_ITER2");
	if (e && e[0] == '1') return "SVG_REF_ITER2=1";
	if (gc->config.is_BAM_output && gc->config.sort_reads_by_coordinates) return "BAM output sorted by coordinate";
	if (gc->config.space_type != GENE_SPACE_BASE || gc->config.convert_color_to_base) return "colour space";
	if (gc->config.do_fusion_detection || gc->config.do_long_del_detection) return "fusion / long-deletion detection";
	if (gc->exonic_region_bitmap) return "exon scoring from an annotation";
	if (gc->config.scRNA_input_mode) return "scRNA input";
	if (gc->config.do_big_margin_filtering_for_reads) return "big-margin read filtering";
	if (gc->input_reads.first_read_file.file_type == GENE_INPUT_BCL) return "BCL input";
	if (svg_rc.complete != 1) return "the chunk's read cache is not complete";
	if ((subread_read_number_t)svg_rc.n != gc->processed_reads_in_chunk) return "the read cache holds another chunk";
	if (memcmp(&svg_rc.start1, &gc->current_circle_start_position_file1, sizeof svg_rc.start1)) return "the chunk starts elsewhere";
	return NULL;
}

static int svg_it2_setup(global_context_t *gc)
{
	if (svg_it2) return 0;
	int rc = svg_gen_setup(gc);
	if (rc) return rc;
	svg_realign_params p;
	memset(&p, 0, sizeof p);
	p.paired = gc->input_reads.is_paired_end_reads;
	p.multi_best = gc->config.multi_best_reads;
	p.reported_multi_best = gc->config.reported_multi_best_reads;
	p.report_multi_mapping = gc->config.report_multi_mapping_reads;
	p.min_votes_first = gc->config.minimum_subread_for_first_read;
	p.min_votes_second = gc->config.minimum_subread_for_second_read;
	p.experiment_type = gc->config.experiment_type;
	p.max_mismatch_exonic = gc->config.max_mismatch_exonic_reads;
	p.max_mismatch_junction = gc->config.max_mismatch_junction_reads;
	p.min_mapped_fraction = gc->config.min_mapped_fraction;
	p.show_soft_clipping = gc->config.show_soft_cliping;
	p.realignment_minimum_variant_distance = gc->config.realignment_minimum_variant_distance;
	p.limited_tree_scan = gc->config.limited_tree_scan;
	p.maximise_sensitivity_indel = gc->config.maximise_sensitivity_indel;
	p.minimum_exonic_subread_fraction = gc->config.minimum_exonic_subread_fraction;
	p.no_tlen_preference = gc->config.no_TLEN_preference;
	p.min_pair_distance = gc->config.minimum_pair_distance;
	p.max_pair_distance = gc->config.maximum_pair_distance;
	p.is_first_read_reversed = gc->config.is_first_read_reversed;
	p.is_second_read_reversed = gc->config.is_second_read_reversed;
	p.do_breakpoint_detection = gc->config.do_breakpoint_detection;
	p.ignore_unmapped_reads = gc->config.ignore_unmapped_reads;
	p.phred_offset = gc->config.phred_score_format == FASTQ_PHRED64 ? 64 : 33;
	{   /* (the tag the reference writes is cut at 310 bytes anyway, core.c:2053) */
		const size_t rg = strnlen(gc->config.read_group_id, sizeof p.read_group_id - 1);
		memcpy(p.read_group_id, gc->config.read_group_id, rg);
		p.read_group_id[rg] = 0;
	}
	return svg_realign_create(svg_gen, &p, &svg_it2);
}

/* chromosome_event_t -> svg_event: the fields iteration two and the anti-supporting read scan
 * read (a calloc'd array of ic->total_events entries, NULL when out of memory) */
static svg_event *svg_events_from_gc(global_context_t *gc, int64_t *n_out)
{
	indel_context_t *ic = (indel_context_t *)gc->module_contexts[MODULE_INDEL_ID];
	int64_t n = ic->total_events, i;
	svg_event *ev = calloc((size_t)(n ? n : 1), sizeof(svg_event));
	*n_out = n;
	if (!ev) return NULL;
	for (i = 0; i < n; i++) {
		const chromosome_event_t *e = ic->event_space_dynamic + i;
		svg_event *o = &ev[i];
		o->small_side = e->event_small_side;
		o->large_side = e->event_large_side;
		o->indel_length = e->indel_length;
		o->junction_flanking_left = e->junction_flanking_left;
		o->junction_flanking_right = e->junction_flanking_right;
		o->indel_at_junction = e->indel_at_junction;
		o->is_negative_strand = e->is_negative_strand;
		o->is_strand_jumped = e->is_strand_jumped;
		o->is_donor_found_or_annotation = e->is_donor_found_or_annotation;
		o->small_side_increasing_coordinate = e->small_side_increasing_coordinate;
		o->large_side_increasing_coordinate = e->large_side_increasing_coordinate;
		o->connected_next_event_distance = e->connected_next_event_distance;
		o->connected_previous_event_distance = e->connected_previous_event_distance;
		o->supporting_reads = e->supporting_reads;
		o->anti_supporting_reads = e->anti_supporting_reads;
		o->final_counted_reads = e->final_counted_reads;
		o->final_reads_mismatches = e->final_reads_mismatches;
		o->event_type = e->event_type;
		o->critical_read_id = e->critical_read_id;
		o->event_quality = e->event_quality;
		o->critical_supporting_reads = e->critical_supporting_reads;
	}
	return ev;
}

static int svg_it2_events_in(global_context_t *gc)
{
	int64_t n;
	svg_event *ev = svg_events_from_gc(gc, &n);
	if (!ev) return SVG_E_NOMEM;
	int rc = svg_realign_set_events(svg_it2, ev, n);
	free(ev);
	return rc;
}

/*
 * anti_supporting_read_scan (core-indel.c:177-330), weakened in the drop-in build like do_voting:
 * the chunk's merged event table and its bigtable records go through svg_events_anti_support
 * (sorted side lists, one binary search per record side, threads over reads); the counts come back
 * into the reference's table.  Fusion / long-deletion detection and colour space keep the
 * reference's scan (ref_anti_supporting_read_scan, the alias oracle/Makefile adds), as does
 * SVG_REF_ANTI=1.
 */
int ref_anti_supporting_read_scan(global_context_t *gc);
void ref_remove_neighbour(global_context_t *gc);
static svg_events *svg_anti_t;   /* the chunk's table after the library's scan, for remove_neighbour */

static int svg_anti_supported(global_context_t *gc)
{
	const char *env = getenv("SVG_REF_ANTI");
	return !(env && env[0] == '1') && !gc->config.do_fusion_detection && !gc->config.do_long_del_detection &&
	       gc->config.space_type == GENE_SPACE_BASE && gc->config.multi_best_reads <= 3 &&
	       !(gc->config.do_remove_neighbour_for_scRNA && gc->config.scRNA_input_mode);
}

int anti_supporting_read_scan(global_context_t *gc)
{
	indel_context_t *ic = (indel_context_t *)gc->module_contexts[MODULE_INDEL_ID];
	if (svg_t_mark > 0) { svg_t_to_anti += miltime() - svg_t_mark; svg_t_mark = 0; }
	if (svg_anti_t) { svg_events_destroy(svg_anti_t); svg_anti_t = NULL; }
	if (!svg_anti_supported(gc)) {
		svg_stage(ST_ANTI, "configuration (SVG_REF_ANTI=1, fusion / long-deletion detection, colour space, -B > 3 or scRNA)");
		return ref_anti_supporting_read_scan(gc);
	}
	if (ic->total_events < 1) {
		svg_stage(ST_ANTI, NULL);
		return 0;
	}
	const double t0 = miltime();
	int64_t n, i;
	int rc = 0;
	svg_event *ev = svg_events_from_gc(gc, &n);
	svg_events *t = NULL;
	if (!ev) rc = SVG_E_NOMEM;
	if (!rc) rc = svg_events_create(&t);
	if (!rc) rc = svg_events_load(t, ev, n);
	if (!rc) {
		svg_params p;
		svg_event_params ep;
		svg_fill_params(gc, &p);
		svg_event_params_default(&ep);
		ep.report_multi_mapping_reads = gc->config.report_multi_mapping_reads;
		rc = svg_events_anti_support(t, &p, &ep, (uint64_t)gc->processed_reads_in_chunk, 1 + gc->input_reads.is_paired_end_reads,
		                             (const svg_mapping_result *)_global_retrieve_alignment_ptr(gc, 0, 0, 0));
	}
	if (!rc && svg_events_count(t) != n) rc = SVG_E_ARG;
	if (!rc) rc = svg_events_get(t, ev);
	for (i = 0; !rc && i < n; i++) ic->event_space_dynamic[i].anti_supporting_reads = ev[i].anti_supporting_reads;
	if (!rc) svg_anti_t = t;   /* remove_neighbour, next, starts from it */
	else if (t) svg_events_destroy(t);
	free(ev);
	svg_t_anti += miltime() - t0;
	if (rc) {
		/* nothing was written back: the reference's own scan on its untouched table */
		char why[300];
		snprintf(why, sizeof why, "library error %d: %s", rc, svg_last_error());
		SUBREADprintf("svg anti-supporting read scan: %s (the reference's scan instead)\n", why);
		svg_stage(ST_ANTI, why);
		return ref_anti_supporting_read_scan(gc);
	}
	svg_stage(ST_ANTI, NULL);
	return 0;
}

static int svg_it2_events_out(global_context_t *gc)
{
	indel_context_t *ic = (indel_context_t *)gc->module_contexts[MODULE_INDEL_ID];
	int64_t n = ic->total_events, i;
	svg_event *ev = calloc((size_t)(n ? n : 1), sizeof(svg_event));
	if (!ev) return SVG_E_NOMEM;
	int rc = svg_realign_get_events(svg_it2, ev);
	for (i = 0; !rc && i < n; i++) {
		chromosome_event_t *e = ic->event_space_dynamic + i;
		e->final_counted_reads = ev[i].final_counted_reads;
		e->junction_flanking_left = ev[i].junction_flanking_left;
		e->junction_flanking_right = ev[i].junction_flanking_right;
	}
	free(ev);
	return rc;
}

/*
 * remove_neighbour (core-indel.c:447-595), weakened like anti_supporting_read_scan: the decisions
 * come from svg_events_remove_neighbour on the table the library's scan just counted (pinned to
 * the reference's own removals, §5e of DESIGN.md), and each newly removed event is then taken
 * out of the reference's site lists (event_entry_table) and typed CHRO_EVENT_TYPE_REMOVED exactly
 * as the reference's removal loop does (core-indel.c:569-593) -- the VCF / BED writers and any
 * later pass see the reference's own state.
 */
void remove_neighbour(global_context_t *gc)
{
	indel_context_t *ic = (indel_context_t *)gc->module_contexts[MODULE_INDEL_ID];
	svg_events *t = svg_anti_t;
	svg_anti_t = NULL;
	if (!t && svg_anti_supported(gc) && ic->total_events < 1) {   /* (an empty table: nothing to remove) */
		svg_stage(ST_RN, NULL);
		return;
	}
	if (!svg_anti_supported(gc) || !t || svg_events_count(t) != ic->total_events) {
		char why[200];
		snprintf(why, sizeof why, "%s (library table %s, %lld vs %lld events)", svg_anti_supported(gc) ? "no library table" : "configuration",
		         t ? "present" : "absent", (long long)(t ? svg_events_count(t) : -1), (long long)ic->total_events);
		svg_stage(ST_RN, why);
		if (t) svg_events_destroy(t);
		ref_remove_neighbour(gc);
		return;
	}
	const double t0 = miltime();
	const int64_t n = ic->total_events;
	svg_event *ev = calloc((size_t)(n ? n : 1), sizeof(svg_event));
	int rc = ev ? svg_events_remove_neighbour(t) : SVG_E_NOMEM;
	if (!rc) rc = svg_events_get(t, ev);
	svg_events_destroy(t);
	if (rc) {
		free(ev);
		char why[300];
		snprintf(why, sizeof why, "library error %d: %s", rc, svg_last_error());
		svg_stage(ST_RN, why);
		ref_remove_neighbour(gc);   /* the table is untouched: the reference decides */
		return;
	}
	svg_stage(ST_RN, NULL);
	HashTable *event_table = ic->event_entry_table;
	chromosome_event_t *event_space = ic->event_space_dynamic;
	for (int64_t no = 0; no < n; no++) {
		chromosome_event_t *del = &event_space[no];
		if (ev[no].event_type != CHRO_EVENT_TYPE_REMOVED || del->event_type == CHRO_EVENT_TYPE_REMOVED) continue;
		for (int side = 0; side < 2; side++) {
			const unsigned int pos = side ? del->event_large_side : del->event_small_side;
			unsigned int *res = HashTableGet(event_table, NULL + pos);
			if (!res) continue;
			const int cur = res[0] & 0x0fffffff;
			int w = 1;
			for (int k = 1; k < cur + 1; k++) {
				if (!res[k]) break;
				if ((int64_t)res[k] - 1 == no) continue;
				if (w != k) res[w] = res[k];
				w++;
			}
			if (w < cur + 1) res[w] = 0;
		}
		if (del->event_type == CHRO_EVENT_TYPE_INDEL && del->inserted_bases) free(del->inserted_bases);
		del->event_type = CHRO_EVENT_TYPE_REMOVED;
	}
	free(ev);
	svg_t_anti += miltime() - t0;
	svg_t_mark = miltime();
}

static int svg_iteration_two(global_context_t *gc, thread_context_t *tc)
{
	double t0 = miltime();
	if (svg_t_mark > 0) { svg_t_to_it2 += t0 - svg_t_mark; svg_t_mark = 0; }
	int rc = svg_it2_setup(gc);
	if (!rc) rc = svg_it2_events_in(gc);
	const int ends = 1 + gc->input_reads.is_paired_end_reads;
	const uint64_t n = svg_rc.n;
	uint64_t *offs = NULL;
	uint16_t *lens = NULL;
	if (!rc) {
		offs = malloc(sizeof(uint64_t) * 3 * (n * ends + 1));
		lens = malloc(sizeof(uint16_t) * (n * ends + 1));
		if (!offs || !lens) rc = SVG_E_NOMEM;
	}
	if (!rc) {
		uint64_t r;
		int e;
		for (r = 0; r < n; r++)
			for (e = 0; e < ends; e++) {
				const uint64_t k = r * ends + e, at = svg_rc.at[r * 2 + e];
				const int rl = svg_rc.rl[r * 2 + e];
				offs[k] = at;
				offs[n * ends + k] = at + strlen(svg_rc.buf + at) + 1;
				offs[2 * n * ends + k] = offs[n * ends + k] + (uint64_t)rl + 1;
				lens[k] = (uint16_t)rl;
			}
	}
	svg_sam_writer *sink = NULL;
	if (!rc) {
		/* SAM: the ordered sink on output_sam_fp.  BAM (the default output): the same sink in BAM mode
		 * on the BAM file, whose blocks are cut where the reference's ordered stream (-T 1 or
		 * --keepReadOrder, writer id -1, core.c:1859-1865,2144-2151) cuts them; without
		 * --keepReadOrder the reference's threads write unordered blocks (core.c:1849-1853), and the
		 * ordered stream holds the same records */
		pthread_mutex_lock(&svg_sam_mu);
		if (!svg_sam) {
			if (gc->config.is_BAM_output) {
				svg_bam_w = gc->output_bam_writer;
				rc = svg_sam_writer_open_bam(svg_bam_w->bam_fp, gc->input_reads.is_paired_end_reads, 1, &svg_sam);
			}
			else rc = svg_sam_writer_open(gc->output_sam_fp, &svg_sam);
			if (rc) rc = SVG_E_IO;
		}
		if (!rc) {
			rc = svg_sam_writer_begin_chunk(svg_sam, (int64_t)n);
			gc->last_written_fragment_number = -2;
			sink = svg_sam;
		}
		pthread_mutex_unlock(&svg_sam_mu);
	}
	if (!rc) {
		svg_fragment_reads R = {svg_rc.buf, offs, offs + n * ends, offs + 2 * n * ends, lens, n};
		svg_realign_stats st;
		memset(&st, 0, sizeof st);
		const unsigned int tlen_n0 = gc->expected_TLEN_read_numbers;
		svg_realign_set_tlen_state(svg_it2, gc->expected_TLEN_read_numbers, (int64_t)gc->expected_TLEN_sum);
		rc = svg_realign_chunk(svg_it2, &R, (svg_mapping_result *)_global_retrieve_alignment_ptr(gc, 0, 0, 0), sink, NULL, NULL,
		                       gc->config.all_threads, &st);
		int64_t tn, ts;
		svg_realign_get_tlen_state(svg_it2, &tn, &ts);
		gc->expected_TLEN_read_numbers = (unsigned int)tn;
		gc->expected_TLEN_sum = (unsigned long long)ts;
		if (tlen_n0 < READPAIRS_FOR_CALC_EXPT_TLEN && tn >= READPAIRS_FOR_CALC_EXPT_TLEN)
			print_in_box(80, 0, 0, "  Estimated fragment length : %d bp\n", (int)(gc->expected_TLEN_sum / gc->expected_TLEN_read_numbers));
		if (!rc) rc = svg_it2_events_out(gc);
#define SVG_ADD(f) do { if (tc) tc->f += st.f; else gc->f += st.f; } while (0)
		SVG_ADD(all_mapped_reads); SVG_ADD(all_correct_PE_reads); SVG_ADD(not_properly_pairs_wrong_arrangement);
		SVG_ADD(not_properly_pairs_different_chro); SVG_ADD(not_properly_different_strands); SVG_ADD(not_properly_pairs_TLEN_wrong);
		SVG_ADD(all_unmapped_reads); SVG_ADD(not_properly_pairs_only_one_end_mapped); SVG_ADD(all_multimapping_reads);
		SVG_ADD(all_uniquely_mapped_reads);
#undef SVG_ADD
	}
	free(offs);
	free(lens);
	if (rc) {
		SUBREADprintf("svg iteration two: %s\n", svg_last_error());
		gc->output_sam_is_full = 1;
	}
	svg_t_realign += miltime() - t0;
	return 0;
}

int do_iteration_two(global_context_t *gc, thread_context_t *tc)
{
	const char *why = svg_it2_unsupported(gc);
	if (!tc || tc->thread_id == 0) svg_stage(ST_IT2, why);
	if (why) return ref_do_iteration_two(gc, tc);
	if (tc && tc->thread_id != 0) return 0;
	return svg_iteration_two(gc, tc);
}

/*
 * The handles are opened on a thread of their own at the first voting run, so that loading the
 * index into HBM (svg_index_open: ~1.9 s for a 3 Gbp index) overlaps the first chunk's read;
 * vote_stage joins it before the first vote.  SVG_DEVICES=0,1,...: one handle per listed device (a
 * device may repeat: several replicas on one GPU); else SVG_DEVICE (default 0).
 */
static pthread_t svg_open_th;
static int svg_open_state;            /* 0 not started, 1 running, 2 joined */
static int svg_open_rc;
static global_context_t *svg_open_gc;

static void *svg_open_run(void *v)
{
	(void)v;
	global_context_t *gc = svg_open_gc;
	const char *ds = getenv("SVG_DEVICES"), *d = getenv("SVG_DEVICE");
	if (ds && ds[0]) {
		int devs[SVG_MAX_DEV], n = 0;
		const char *q = ds;
		while (*q && n < SVG_MAX_DEV) {
			devs[n++] = atoi(q);
			while (*q && *q != ',') q++;
			if (*q == ',') q++;
		}
		svg_open_rc = svg_attach_devices(gc, devs, n);
	} else svg_open_rc = svg_attach(gc, d ? atoi(d) : 0);
	return NULL;
}

/* the handles, open (thread 0 of the voting run, before its first vote) */
static int svg_open_join(void)
{
	pthread_mutex_lock(&svg_sam_mu_init);
	if (svg_open_state == 1) {
		pthread_join(svg_open_th, NULL);
		svg_open_state = 2;
	}
	const int rc = svg_open_rc;
	pthread_mutex_unlock(&svg_sam_mu_init);
	return rc;
}

int do_voting(global_context_t *gc, thread_context_t *tc)
{
	pthread_mutex_lock(&svg_sam_mu_init);
	if (svg_open_state == 0) {
		svg_open_gc = gc;
		if (pthread_create(&svg_open_th, NULL, svg_open_run, NULL) == 0) svg_open_state = 1;
		else {
			svg_open_run(NULL);
			svg_open_state = 2;
		}
	}
	pthread_mutex_unlock(&svg_sam_mu_init);
	if (!tc || gc->config.all_threads < 2) return do_voting_gpu(gc, tc);
	return do_voting_gpu_mt(gc, tc, gc->config.all_threads);
}
#endif
