/*
 * svg_host.c -- host C side of the vote path: error text, parameter defaults,
 * and the loader that turns the reference's on-disk index into the flat
 * arrays uploaded to HBM.
 *
 *   .tab   gehash_load      sorted-hashtable.c:1390-1625   ("2subindx", option
 *          TLVs 0x0101 gap / 0x0102 padding, i64 items, i32 nb, then per bucket
 *          i32 n, i32 space, i16 keys[n], u32 values[n], then u8 is_small)
 *   .array gvindex_load     gene-value-index.c:190-228
 *   .reads load_offsets     gene-algorithms.c:1293-1370
 *
 * The .tab is mmap'ed; one sequential pass over the bucket headers yields the
 * bucket offsets, then worker threads copy disjoint bucket ranges.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdarg.h>
#include <pthread.h>
#include <fcntl.h>
#include <unistd.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include "svg_internal.h"

static double t_now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static __thread char g_err[1024];

void svg_set_error(const char *fmt, ...)
{
	va_list ap;
	va_start(ap, fmt);
	vsnprintf(g_err, sizeof g_err, fmt, ap);
	va_end(ap);
}

const char *svg_last_error(void) { return g_err; }
int svg_abi_version(void) { return SVG_ABI_VERSION; }

/* Implementation options (include/subread_vote.h): explicit, process-wide, never read from the
 * environment, and none of them changes a record. */
static struct { const char *name; volatile int64_t value; } g_opts[] = {
	{"host_threads", 0}, {"host_sub", 0}, {"host_ramp", 1}, {"chunk", 0}, {"overlap", -1},
	{"lane", 0}, {"lane_unfused", 0}, {"lane_cap", 0},
	{"no_bcode", 0}, {"no_khash", 0}, {"khash64", 0}, {"no_bline", 0}, {"no_compact", 0}, {"keys_literal", 0},
	{"wave_cap", -1}, {"wave_static", -1}, {"probe_cap", 0}, {"long_probes", 0}, {"dev_pace", 0},
	{"debug", 0},   /* bits: 1 vote-path batches, 2 host pipeline, 4 sublong chunks, 8 index load, 16 iteration two */
};
#define N_OPTS ((int)(sizeof g_opts / sizeof g_opts[0]))

int svg_set_option(const char *name, int64_t value)
{
	for (int i = 0; name && i < N_OPTS; i++)
		if (!strcmp(g_opts[i].name, name)) { g_opts[i].value = value; return 0; }
	svg_set_error("unknown option '%s'", name ? name : "(null)");
	return SVG_E_ARG;
}

int64_t svg_get_option(const char *name)
{
	for (int i = 0; name && i < N_OPTS; i++)
		if (!strcmp(g_opts[i].name, name)) return g_opts[i].value;
	return 0;
}

/* init_global_context (core-indel.c:4399-4538) -> parse_opts_* -> load_global_context (core.c:4075-4094) */
void svg_params_default(svg_params *p, int program, int paired_end)
{
	memset(p, 0, sizeof *p);
	p->total_subreads = 10;
	p->min_votes_first = 3;
	p->min_votes_second = 1;
	p->max_indel_length = 5;
	p->top_scores = 3;
	p->min_pair_distance = 50;
	p->max_pair_distance = 600;
	p->reverse_r1 = 0;
	p->reverse_r2 = 1;
	p->big_margin_record_size = 9;
	p->maximum_intron_length = 500000;
	p->prefer_donor_receptor_junctions = 1;
	p->check_donor_at_junctions = 1;
	p->max_insertion_at_junctions = 0;
	if (program == SVG_PROGRAM_SUBJUNC) {          /* core-interface-subjunc.c:268-282 */
		p->do_breakpoint_detection = 1;
		p->total_subreads = 14;
		p->min_votes_first = 1;
		p->min_votes_second = 1;
		p->do_big_margin_filtering_for_junctions = 1;
	}
	p->more_accurate_fusions = 0;                  /* no fusion/long-del: core-interface-*.c:648/671 */
	p->max_vote_combinations = 3;                  /* core.c:4075-4084 */
	p->multi_best = 3;
	p->max_vote_simples = paired_end ? 64 : 3;
	p->max_vote_number_cutoff = 2;
}

/* ------------------------------------------------------------------ index loader */
typedef struct {
	const uint8_t *base;
	const uint64_t *hdr_off;   /* file offset of each bucket header */
	svg_host_index *ix;
	uint32_t b0, b1;
} copy_job;

static void *copy_worker(void *arg)
{
	copy_job *j = arg;
	uint32_t b;
	for (b = j->b0; b < j->b1; b++) {
		uint32_t n = j->ix->bstart[b + 1] - j->ix->bstart[b];
		const uint8_t *h = j->base + j->hdr_off[b] + 8;
		if (!n) continue;
		memcpy(j->ix->keys + j->ix->bstart[b], h, 2 * (size_t)n);
		memcpy(j->ix->vals + j->ix->bstart[b], h + 2 * (size_t)n, 4 * (size_t)n);
	}
	return NULL;
}

void svg_host_index_free(svg_host_index *ix)
{
	if (!ix) return;
	free(ix->bstart); free(ix->keys); free(ix->vals); free(ix->values);
	free(ix->chr_end); free(ix->chr_name);
	if (ix->map) munmap(ix->map, ix->map_len);
	memset(ix, 0, sizeof *ix);
}

static int load_tab(const char *fn, svg_host_index *ix, int threads)
{
	int fd = open(fn, O_RDONLY);
	struct stat st;
	const uint8_t *m, *p, *end;
	uint64_t *hdr = NULL, cur = 0;
	uint32_t b;
	if (fd < 0) { svg_set_error("index table '%s' not found", fn); return SVG_E_IO; }
	if (fstat(fd, &st) || st.st_size < 32) { close(fd); svg_set_error("index table '%s' unreadable", fn); return SVG_E_IO; }
	const int dbg = (svg_get_option("debug") & 8) != 0;
	double t0 = t_now();
	ix->map_len = st.st_size;
	ix->map = mmap(NULL, ix->map_len, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
	close(fd);
	if (ix->map == MAP_FAILED) { ix->map = NULL; svg_set_error("mmap of '%s' failed", fn); return SVG_E_IO; }
	m = ix->map; end = m + ix->map_len;
	if (memcmp(m, "2subindx", 8)) { svg_set_error("'%s' is not a v2 subread index (magic)", fn); return SVG_E_FORMAT; }
	p = m + 8;
	for (;;) {
		int16_t k, l;
		if (p + 2 > end) return SVG_E_FORMAT;
		memcpy(&k, p, 2); p += 2;
		if (!k) break;
		memcpy(&l, p, 2); p += 2;
		if (k == 0x0101) { int16_t v; memcpy(&v, p, 2); ix->gap = v; }
		else if (k == 0x0102) { int16_t v; memcpy(&v, p, 2); ix->padding = v; }
		p += l;
	}
	{
		int64_t items; int32_t nb;
		memcpy(&items, p, 8); p += 8;
		memcpy(&nb, p, 4); p += 4;
		if (items < 1 || (uint64_t)items > 0xffffffffull || nb < 1) { svg_set_error("'%s': bad item/bucket count", fn); return SVG_E_FORMAT; }
		ix->items = items; ix->nb = nb;
	}
	if (ix->gap < 1) { svg_set_error("'%s': no index gap option", fn); return SVG_E_FORMAT; }
	ix->bstart = malloc(sizeof(uint32_t) * ((size_t)ix->nb + 1));
	hdr = malloc(sizeof(uint64_t) * ix->nb);
	ix->keys = malloc(2 * ix->items + 64);
	ix->vals = malloc(4 * ix->items + 64);
	if (!ix->bstart || !hdr || !ix->keys || !ix->vals) { free(hdr); svg_set_error("out of host memory loading index"); return SVG_E_NOMEM; }
	const double t1 = t_now();
	for (b = 0; b < ix->nb; b++) {
		int32_t n;
		if (p + 8 > end) { free(hdr); svg_set_error("'%s' truncated", fn); return SVG_E_FORMAT; }
		memcpy(&n, p, 4);
		hdr[b] = (uint64_t)(p - m);
		ix->bstart[b] = (uint32_t)cur;
		cur += (uint32_t)n;
		p += 8 + 6 * (size_t)(uint32_t)n;
	}
	ix->bstart[ix->nb] = (uint32_t)cur;
	if (cur != ix->items || p > end) { free(hdr); svg_set_error("'%s': bucket sizes do not add up", fn); return SVG_E_FORMAT; }
	const double t2 = t_now();
	{
		int t, nt = threads < 1 ? 1 : (threads > 64 ? 64 : threads);
		pthread_t th[64];
		copy_job jb[64];
		for (t = 0; t < nt; t++) {
			jb[t].base = m; jb[t].hdr_off = hdr; jb[t].ix = ix;
			jb[t].b0 = (uint32_t)((uint64_t)ix->nb * t / nt);
			jb[t].b1 = (uint32_t)((uint64_t)ix->nb * (t + 1) / nt);
			if (pthread_create(&th[t], NULL, copy_worker, &jb[t])) { copy_worker(&jb[t]); th[t] = 0; }
		}
		for (t = 0; t < nt; t++)
			if (th[t]) pthread_join(th[t], NULL);   /* 0: that range ran inline */
	}
	free(hdr);
	const double t3 = t_now();
	munmap(ix->map, ix->map_len);
	ix->map = NULL;
	if (dbg)
		fprintf(stderr, "[svg] load_tab %s: %.2f GB, mmap+populate %.3f s, bucket headers %.3f s, copy (%d threads) %.3f s, unmap %.3f s\n",
		        fn, (double)ix->map_len / 1e9, t1 - t0, t2 - t1, threads, t3 - t2, t_now() - t3);
	return 0;
}

/* index blocks <prefix>.00.b.tab, .01.b.tab, ... (load_global_context counts them the same
 * way, core.c:4193-4205) */
int svg_index_count_blocks(const char *prefix)
{
	char fn[4096];
	int n = 0;
	for (;;) {
		snprintf(fn, sizeof fn, "%s.%02d.b.tab", prefix, n);
		if (access(fn, F_OK) != 0) break;
		n++;
	}
	return n;
}

/* The .tab of a block mapped for a streaming load (svg_vote.hip index_open_block): the header
 * (options, items, buckets) parsed, *first = the first bucket header.  Bucket b's header is then at
 * first + 8 b + 6 bstart[b] (header {i32 n, i32 space}, then i16 keys[n], u32 vals[n]). */
int svg_tab_map(const char *fn, svg_host_index *ix, const uint8_t **first)
{
	int fd = open(fn, O_RDONLY);
	struct stat st;
	if (fd < 0) { svg_set_error("index table '%s' not found", fn); return SVG_E_IO; }
	if (fstat(fd, &st) || st.st_size < 32) { close(fd); svg_set_error("index table '%s' unreadable", fn); return SVG_E_IO; }
	ix->map_len = st.st_size;
	ix->map = mmap(NULL, ix->map_len, PROT_READ, MAP_PRIVATE, fd, 0);
	close(fd);
	if (ix->map == MAP_FAILED) { ix->map = NULL; svg_set_error("mmap of '%s' failed", fn); return SVG_E_IO; }
	madvise(ix->map, ix->map_len, MADV_SEQUENTIAL);
	const uint8_t *m = ix->map, *p = m + 8, *end = m + ix->map_len;
	if (memcmp(m, "2subindx", 8)) { svg_set_error("'%s' is not a v2 subread index (magic)", fn); return SVG_E_FORMAT; }
	for (;;) {
		int16_t k, l;
		if (p + 4 > end) { svg_set_error("'%s' truncated", fn); return SVG_E_FORMAT; }
		memcpy(&k, p, 2); p += 2;
		if (!k) break;
		memcpy(&l, p, 2); p += 2;
		if (k == 0x0101) { int16_t v; memcpy(&v, p, 2); ix->gap = v; }
		else if (k == 0x0102) { int16_t v; memcpy(&v, p, 2); ix->padding = v; }
		p += l;
	}
	int64_t items; int32_t nb;
	if (p + 12 > end) { svg_set_error("'%s' truncated", fn); return SVG_E_FORMAT; }
	memcpy(&items, p, 8); p += 8;
	memcpy(&nb, p, 4); p += 4;
	if (items < 1 || (uint64_t)items > 0xffffffffull || nb < 1) { svg_set_error("'%s': bad item/bucket count", fn); return SVG_E_FORMAT; }
	if (ix->gap < 1) { svg_set_error("'%s': no index gap option", fn); return SVG_E_FORMAT; }
	ix->items = items; ix->nb = nb;
	*first = p;
	return 0;
}

/* one block's .array and the chromosome table of <prefix>.reads (gvindex_load, load_offsets) */
static int load_meta(const char *prefix, int block, svg_host_index *ix);

int svg_host_index_load_meta(const char *prefix, int block, svg_host_index *ix)
{
	return load_meta(prefix, block, ix);   /* (on an error the caller frees ix: the .tab may still be mapped) */
}

/* one block: <prefix>.NN.b.tab and .NN.b.array (gehash_load / gvindex_load of read_chunk_circles,
 * core.c:3553-3582), plus the chromosome table of <prefix>.reads, into host arrays */
int svg_host_index_load_block(const char *prefix, int block, svg_host_index *ix, int threads)
{
	char fn[4096];
	int rc;
	memset(ix, 0, sizeof *ix);
	snprintf(fn, sizeof fn, "%s.%02d.b.tab", prefix, block);
	rc = load_tab(fn, ix, threads);
	if (rc) { svg_host_index_free(ix); return rc; }
	rc = load_meta(prefix, block, ix);
	if (rc) svg_host_index_free(ix);
	return rc;
}

typedef struct { int fd; uint8_t *dst; size_t len; off_t off; size_t got; } pread_job;
static void *pread_run(void *v)
{
	pread_job *j = v;
	while (j->got < j->len) {
		const ssize_t r = pread(j->fd, j->dst + j->got, j->len - j->got, j->off + (off_t)j->got);
		if (r <= 0) break;
		j->got += (size_t)r;
	}
	return NULL;
}
/* len bytes of fd at off into dst with `threads` preads; the bytes read before the first short slice */
static size_t pread_parallel(int fd, uint8_t *dst, size_t len, off_t off, int threads)
{
	pread_job jobs[16];
	pthread_t th[16];
	int started[16];
	if (threads > 16) threads = 16;
	for (int t = 0; t < threads; t++) {
		const size_t a = len * (size_t)t / (size_t)threads, b = len * (size_t)(t + 1) / (size_t)threads;
		jobs[t] = (pread_job){fd, dst + a, b - a, off + (off_t)a, 0};
		started[t] = pthread_create(&th[t], NULL, pread_run, &jobs[t]) == 0;
		if (!started[t]) pread_run(&jobs[t]);
	}
	size_t got = 0;
	int short_seen = 0;
	for (int t = 0; t < threads; t++) {
		if (started[t]) pthread_join(th[t], NULL);
		if (!short_seen) got += jobs[t].got;
		if (jobs[t].got < jobs[t].len) short_seen = 1;
	}
	return got;
}

static int load_meta(const char *prefix, int block, svg_host_index *ix)
{
	char fn[4096];
	FILE *fp;

	snprintf(fn, sizeof fn, "%s.%02d.b.array", prefix, block);
	fp = fopen(fn, "rb");
	if (!fp) { svg_set_error("'%s' not found", fn); return SVG_E_IO; }
	if (fread(&ix->start_point, 4, 1, fp) != 1 || fread(&ix->length, 4, 1, fp) != 1) {
		fclose(fp); svg_set_error("'%s' truncated", fn); return SVG_E_FORMAT;
	}
	ix->start_base_offset = ix->start_point - ix->start_point % 4;
	{
		uint32_t useful = (ix->length + ix->start_point - ix->start_base_offset) >> 2;
		ix->values_bytes = useful + 1;
		ix->values = malloc((size_t)ix->values_bytes + 64);
		if (!ix->values) { fclose(fp); svg_set_error("out of memory"); return SVG_E_NOMEM; }
		/* the packed bases (~750 MB at 3 Gbp) in parallel slices: the page faults of the fresh buffer
		 * and the copies spread over threads (one fread took ~1.7 s beside the .tab's load) */
		const size_t want = (size_t)useful + 1;
		size_t got = 0;
		if (want >= ((size_t)8 << 20)) got = pread_parallel(fileno(fp), ix->values, want, 8, 8);
		else got = fread(ix->values, 1, want, fp);
		if (got < useful) {
			fclose(fp); svg_set_error("'%s' truncated", fn); return SVG_E_FORMAT;
		}
		memset(ix->values + got, 0, ix->values_bytes + 64 - got);
	}
	fclose(fp);

	snprintf(fn, sizeof fn, "%s.reads", prefix);
	fp = fopen(fn, "r");
	if (!fp) { svg_set_error("'%s' not found", fn); return SVG_E_IO; }
	{
		char line[4096];
		uint32_t cap = 64;
		ix->chr_end = malloc(4 * cap);
		ix->chr_name = malloc(sizeof(*ix->chr_name) * cap);
		while (fgets(line, sizeof line, fp)) {
			char *tab;
			size_t L = strlen(line);
			while (L && (line[L - 1] == '\n' || line[L - 1] == '\r')) line[--L] = 0;
			if (L < 2) continue;
			if (ix->n_chr == cap) {
				cap *= 2;
				ix->chr_end = realloc(ix->chr_end, 4 * cap);
				ix->chr_name = realloc(ix->chr_name, sizeof(*ix->chr_name) * cap);
			}
			ix->chr_end[ix->n_chr] = (uint32_t)atoll(line);
			tab = strchr(line, '\t');
			snprintf(ix->chr_name[ix->n_chr], 200, "%s", tab ? tab + 1 : "");
			ix->n_chr++;
		}
	}
	fclose(fp);
	if (!ix->n_chr) { svg_set_error("'%s' is empty", fn); return SVG_E_FORMAT; }
	return 0;
}

int svg_host_index_load(const char *prefix, svg_host_index *ix, int threads)
{
	return svg_host_index_load_block(prefix, 0, ix, threads);
}
