/*
 * svg_realign.c -- iteration two (include/subread_realign.h): realignment of every read end's
 * vote records against the chunk's event table, the choice among a read's (pair's) candidate
 * alignments, and its SAM records.  Restates do_iteration_two (reference core.c:2486-3018) and
 * what it calls; every function cites the lines it follows.  Host C: the reads of a chunk are
 * independent once the event table is fixed, so they are dealt to worker threads in blocks and
 * their SAM text goes to the ordered sink (svg_sam.c) in fragment order.
 *
 * What is done differently from the reference (same results):
 *   - the event site lists are one flat sorted array behind an open-addressing map of
 *     coordinates, built once per chunk as sort_junction_entry_table orders them (core-indel.c:
 *     847-929) with remove_neighbour's removals (core-indel.c:573-593) taken out; a coarse
 *     bitmap (one bit per 64 coordinates, like the reference's byte test in
 *     there_are_events_in_range) skips the lookup where no event side lies;
 *   - match_chro (gene-value-index.c:856-959) compares 16 bases per step: the read's 2-bit codes
 *     (A 0, G 1, C 2, every other character 3, as the function's switch counts them) XOR the
 *     .array's 2-bit LSB-first word, the equal pairs counted with a popcount;
 *   - find_soft_clipping and the mismatch count of final_CIGAR_quality read one per-base match
 *     bitmap of the section (read character == gvindex_get's character), computed the same way;
 *   - final_CIGAR_quality's quality score (a float that only feeds realignment_result_t.
 *     final_quality, which nothing after iteration two reads) is not computed; the mismatch
 *     count it returns is the all-mismatch count the reference assigns at core-junction.c:3148;
 *   - per-thread counters and event support (final_counted_reads, flanking maxima) are summed
 *     after the chunk instead of taken under event_body_locks (sums and maxima: same values).
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <pthread.h>
#include <time.h>
#include "svg_internal.h"

static double now_s(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

#define MAX_EV_READ   8      /* MAX_EVENTS_IN_READ, subread.h:70 */
#define MAX_ALN       2      /* MAX_ALIGNMENT_PER_ANCHOR, subread.h:196 */
#define TOTAL_TRIES   50     /* REALIGN_TOTAL_TRIES, core-junction.h:27 */
#define SITE_MAX      9      /* MAX_EVENT_ENTRIES_PER_SITE, core-indel.h:34 */
#define CIGAR_LEN     110    /* CORE_MAX_CIGAR_STR_LEN, core.h:63 */
#define ADD_INFO_LEN  400    /* CORE_ADDITIONAL_INFO_LENGTH */
#define LONG_READ     160    /* EXON_LONG_READ_LENGTH */
#define MAXRL         1210   /* MAX_READ_LENGTH */
#define TLEN_PAIRS    1000   /* READPAIRS_FOR_CALC_EXPT_TLEN, core.h:65 */
#define EV_INDEL      8
#define EV_JUNCTION   64
#define EV_FUSION     128
#define F_GT_AG       1      /* CORE_IS_GT_AG_DONORS */
#define F_NOTFOUND    2      /* CORE_NOTFOUND_DONORS */
#define F_NEG         8      /* CORE_IS_NEGATIVE_STRAND */
#define F_FULLY       16     /* CORE_IS_FULLY_EXPLAINED */
#define F_BREAKEVEN   32     /* CORE_IS_BREAKEVEN */
#define F_PAIRED_END  128    /* CORE_IS_PAIRED_END */
#define F_TOO_MANY    256    /* CORE_TOO_MANY_MISMATCHES */
#define S_PAIRED      0x01   /* SAM_FLAG_*, subread.h:45-54 */
#define S_PROPER      0x02
#define S_UNMAPPED    0x04
#define S_MATE_UNMAP  0x08
#define S_REVERSE     0x10
#define S_MATE_REV    0x20
#define S_FIRST       0x40
#define S_SECOND      0x80
#define S_SECONDARY   0x100

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int is_digit(int c) { return c >= '0' && c <= '9'; }

void svg_realign_params_default(svg_realign_params *p, int program, int paired, int rna)
{
	memset(p, 0, sizeof *p);
	/* init_global_context (core-indel.c:4399-4538), then the program's own settings
	 * (core-interface-aligner.c:268-276, core-interface-subjunc.c:264-283) */
	p->paired = paired;
	p->multi_best = 1;
	p->reported_multi_best = 1;
	p->min_votes_first = 3;
	p->min_votes_second = 1;
	p->max_mismatch_exonic = 3;
	p->max_mismatch_junction = 3;
	p->show_soft_clipping = 1;
	p->realignment_minimum_variant_distance = 16;
	p->minimum_exonic_subread_fraction = -1.0f;
	p->min_pair_distance = 50;
	p->max_pair_distance = 600;
	p->is_second_read_reversed = 1;
	p->phred_offset = 33;
	if (program == SVG_PROGRAM_SUBJUNC) {
		p->experiment_type = SVG_EXPERIMENT_RNASEQ;
		p->minimum_exonic_subread_fraction = 0.3f;
		p->do_breakpoint_detection = 1;
	} else p->experiment_type = rna ? SVG_EXPERIMENT_RNASEQ : SVG_EXPERIMENT_DNASEQ;
}

/* ------------------------------------------------------------------ the event site lists */
typedef struct { uint32_t key, off; uint32_t n; } site_ent;

struct svg_realign {
	svg_realign_params p;
	const svg_genome_arrays *g;
	svg_event *ev;               /* the chunk's table; realignment support added to its copy */
	int64_t n_ev;
	site_ent *site;              /* coordinate -> ids[off .. off+n) (event ids in list order) */
	uint64_t site_cap;
	uint32_t *ids;
	uint64_t *bm_small, *bm_large;   /* one bit per 64 coordinates: a live small / large side */
	int64_t tlen_n, tlen_sum;
};

#define BM_WORDS (1u << 20)   /* 2^32 coordinates / 64 per bit / 64 bits per word */

static inline int bm_get(const uint64_t *bm, uint32_t pos) { return (int)((bm[pos >> 12] >> ((pos >> 6) & 63)) & 1); }
static inline void bm_set(uint64_t *bm, uint32_t pos) { bm[pos >> 12] |= 1ull << ((pos >> 6) & 63); }

static inline uint64_t site_hash(uint32_t k) { return (k * 0x9E3779B97F4A7C15ull) >> 17; }

static const site_ent *site_find(const svg_realign *ra, uint32_t key)
{
	if (!ra->site_cap) return NULL;
	const uint64_t m = ra->site_cap - 1;
	for (uint64_t i = site_hash(key) & m;; i = (i + 1) & m) {
		if (ra->site[i].n && ra->site[i].key == key) return &ra->site[i];
		if (!ra->site[i].n) return NULL;
	}
}

/* scanning_events_compare, core-indel.c:773-796 */
typedef struct { uint32_t pos; uint32_t id; } scan_rec;
static const svg_event *g_sort_ev;
static int scan_cmp(const void *va, const void *vb)
{
	const scan_rec *a = va, *b = vb;
	if (a->pos != b->pos) return a->pos > b->pos ? 1 : -1;
	const svg_event *l = &g_sort_ev[a->id], *r = &g_sort_ev[b->id];
	const int lk = (l->is_donor_found_or_annotation & 64) != 0, rk = (r->is_donor_found_or_annotation & 64) != 0;
	if (lk != rk) return lk ? 1 : -1;
	if (l->supporting_reads != r->supporting_reads) return l->supporting_reads > r->supporting_reads ? -1 : 1;
	const int al = abs(l->indel_length), ar = abs(r->indel_length);
	if (al != ar) return al < ar ? 1 : -1;
	if (l->indel_length != r->indel_length) return l->indel_length > r->indel_length ? -1 : 1;
	if (l->small_side != r->small_side) return l->small_side > r->small_side ? 1 : -1;
	if (l->large_side != r->large_side) return l->large_side > r->large_side ? 1 : -1;
	return a->id < b->id ? -1 : (a->id > b->id);   /* (the same event twice: never) */
}

static pthread_mutex_t sort_mu = PTHREAD_MUTEX_INITIALIZER;

int svg_realign_set_events(svg_realign *ra, const svg_event *ev, int64_t n)
{
	if (!ra || n < 0 || (n && !ev)) { svg_set_error("svg_realign_set_events: bad argument"); return SVG_E_ARG; }
	free(ra->ev); free(ra->site); free(ra->ids);
	ra->ev = NULL; ra->site = NULL; ra->ids = NULL; ra->site_cap = 0; ra->n_ev = 0;
	memset(ra->bm_small, 0, sizeof(uint64_t) * BM_WORDS);
	memset(ra->bm_large, 0, sizeof(uint64_t) * BM_WORDS);
	if (!n) return 0;
	ra->ev = malloc(sizeof(svg_event) * (size_t)n);
	scan_rec *rec = malloc(sizeof(scan_rec) * 2 * (size_t)n);
	if (!ra->ev || !rec) { free(rec); svg_set_error("out of memory"); return SVG_E_NOMEM; }
	memcpy(ra->ev, ev, sizeof(svg_event) * (size_t)n);
	ra->n_ev = n;
	/* sort_junction_entry_table: both sides of every event of the merged table, sorted by
	 * scanning_events_compare; the first SITE_MAX records of a coordinate make its id list */
	for (int64_t i = 0; i < n; i++) {
		rec[2 * i].pos = ev[i].small_side; rec[2 * i].id = (uint32_t)i;
		rec[2 * i + 1].pos = ev[i].large_side; rec[2 * i + 1].id = (uint32_t)i;
	}
	pthread_mutex_lock(&sort_mu);
	g_sort_ev = ev;
	qsort(rec, 2 * (size_t)n, sizeof(scan_rec), scan_cmp);
	pthread_mutex_unlock(&sort_mu);
	uint64_t nsites = 0;
	for (int64_t i = 0; i < 2 * n; i++) if (!i || rec[i].pos != rec[i - 1].pos) nsites++;
	ra->site_cap = 16;
	while (ra->site_cap < 2 * nsites + 16) ra->site_cap *= 2;
	ra->site = calloc(ra->site_cap, sizeof(site_ent));
	ra->ids = malloc(sizeof(uint32_t) * 2 * (size_t)n);
	if (!ra->site || !ra->ids) { free(rec); svg_set_error("out of memory"); return SVG_E_NOMEM; }
	uint32_t w = 0;
	for (int64_t i = 0; i < 2 * n;) {
		int64_t j = i;
		while (j < 2 * n && rec[j].pos == rec[i].pos) j++;
		const uint32_t off = w;
		/* the list as HashTablePut stored it, then remove_neighbour's removals (event type 0) */
		for (int64_t k = i; k < j && k < i + SITE_MAX; k++)
			if (ev[rec[k].id].event_type) ra->ids[w++] = rec[k].id;
		if (w > off) {
			const uint64_t m = ra->site_cap - 1;
			uint64_t h = site_hash(rec[i].pos) & m;
			while (ra->site[h].n) h = (h + 1) & m;
			ra->site[h].key = rec[i].pos;
			ra->site[h].off = off;
			ra->site[h].n = w - off;
			for (uint32_t q = off; q < w; q++) {
				const svg_event *e = &ev[ra->ids[q]];
				if (e->small_side == rec[i].pos) bm_set(ra->bm_small, rec[i].pos);
				if (e->large_side == rec[i].pos) bm_set(ra->bm_large, rec[i].pos);
			}
		}
		i = j;
	}
	free(rec);
	return 0;
}

int svg_realign_get_events(const svg_realign *ra, svg_event *out)
{
	if (!ra || (!out && ra->n_ev)) { svg_set_error("svg_realign_get_events: bad argument"); return SVG_E_ARG; }
	if (ra->n_ev) memcpy(out, ra->ev, sizeof(svg_event) * (size_t)ra->n_ev);
	return 0;
}

void svg_realign_set_tlen_state(svg_realign *ra, int64_t read_numbers, int64_t sum) { ra->tlen_n = read_numbers; ra->tlen_sum = sum; }
void svg_realign_get_tlen_state(const svg_realign *ra, int64_t *read_numbers, int64_t *sum)
{
	if (read_numbers) *read_numbers = ra->tlen_n;
	if (sum) *sum = ra->tlen_sum;
}

/* search_event (core-indel.c:1420-1461) by one side, types INDEL | JUNCTION | FUSION */
static int search_side(const svg_realign *ra, uint32_t pos, int large, uint32_t *out)
{
	if (pos < 1 || pos > 0xffff0000u) return 0;
	if (!bm_get(large ? ra->bm_large : ra->bm_small, pos)) return 0;
	const site_ent *s = site_find(ra, pos);
	if (!s) return 0;
	int n = 0;
	for (uint32_t k = 0; k < s->n; k++) {
		const uint32_t id = ra->ids[s->off + k];
		const svg_event *e = &ra->ev[id];
		if (!(e->event_type & (EV_INDEL | EV_JUNCTION | EV_FUSION))) continue;
		if ((large ? e->large_side : e->small_side) != pos) continue;
		out[n++] = id;
	}
	return n;
}

/* there_are_events_in_range (core-indel.c:1339-1357) as a filter: any live side in
 * [pos, pos + len] at the bitmap's granularity */
static int events_in_range(const uint64_t *bm, uint32_t pos, int len)
{
	/* the same byte range as the reference: bytes (pos >> 6) .. ((pos + len) >> 6) inclusive,
	 * 32-bit unsigned arithmetic; one bit here per byte there */
	const uint32_t a = (pos >> 6) & 0x3ffffffu, b = 1 + (((uint32_t)(pos + (uint32_t)len) >> 6) & 0x3ffffffu);
	for (uint32_t k = a; k < b; k++)
		if ((bm[k >> 6] >> (k & 63)) & 1) return 1;
	return 0;
}

/* ------------------------------------------------------------------ genome / read comparisons */
/* gvindex_get (gene-value-index.c:96-107): 'A' 'G' 'C' 'T' or 'N' past the array */
static inline char gv_char(const garray *a, uint32_t pos)
{
	const uint32_t byte = (pos - a->start_base_offset) >> 2;
	if (byte >= a->values_bytes - 1) return 'N';
	return "AGCT"[(a->values[byte] >> (pos % 4 * 2)) & 3];
}

static inline uint64_t load64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }

/* 16 bases of the array from pos (base k at bits 2k); caller guarantees the bytes exist */
static inline uint32_t gv_word16(const garray *a, uint32_t pos)
{
	const uint32_t rel = pos - a->start_base_offset;
	return (uint32_t)(load64(a->values + (rel >> 2)) >> ((rel & 3) * 2));
}

/* one oriented read text with its 2-bit codes and its non-ACGT mask */
typedef struct {
	char text[MAXRL + 8];
	int len;
	uint64_t code[MAXRL / 32 + 4];   /* base i at bits 2 (i % 32) of code[i / 32]; A0 G1 C2 other 3 */
	uint64_t odd[MAXRL / 64 + 4];    /* bit i: character not one of A C G T */
} rtext;

static uint8_t code_tab[256], odd_tab[256];   /* match_chro's code of a character; not A C G T */

static void rtext_build(rtext *t, const char *s, int len)
{
	memcpy(t->text, s, (size_t)len);
	memset(t->text + len, 0, 8);
	t->len = len;
	const int nw = (len + 31) / 32, no = (len + 63) / 64;
	for (int w = 0; w < nw; w++) {
		uint64_t v = 0;
		const int b = w * 32, e = b + 32 < len ? b + 32 : len;
		for (int i = e - 1; i >= b; i--) v = (v << 2) | code_tab[(unsigned char)s[i]];
		t->code[w] = v;
	}
	for (int w = nw; w < MAXRL / 32 + 4; w++) t->code[w] = 0;
	for (int w = 0; w < no; w++) {
		uint64_t v = 0;
		const int b = w * 64, e = b + 64 < len ? b + 64 : len;
		for (int i = e - 1; i >= b; i--) v = (v << 1) | odd_tab[(unsigned char)s[i]];
		t->odd[w] = v;
	}
	for (int w = no; w < MAXRL / 64 + 4; w++) t->odd[w] = 0;
}

/* 16 read codes from base o (0 <= o, o + 16 <= sizeof code) */
static inline uint32_t rt_word16(const rtext *t, int o)
{
	const int w = o >> 5, s = (o & 31) * 2;
	uint64_t v = t->code[w] >> s;
	if (s) v |= t->code[w + 1] << (64 - s);
	return (uint32_t)v;
}

static inline uint32_t eq_pairs(uint32_t x) { return ~(x | (x >> 1)) & 0x55555555u; }

/* match_chro (gene-value-index.c:856-959), base space, positive strand: the read from offset o,
 * test_len bases at pos */
static int match_chro(const rtext *t, int o, const garray *a, uint32_t pos, int test_len)
{
	if ((uint32_t)(pos + (uint32_t)test_len) >= a->length + a->start_point) return 0;
	if (pos > 0xffff0000u) return 0;
	uint32_t byte = (pos - a->start_base_offset) >> 2;
	if (byte >= a->values_bytes) return 0;
	if (test_len <= 0) return 0;
	const uint64_t last_byte = (uint64_t)byte + ((uint64_t)test_len + 3) / 4 + 1;
	if (o >= 0 && o + test_len <= t->len && last_byte + 9 < a->values_bytes) {
		int ret = 0, i = 0;
		for (; i + 16 <= test_len; i += 16)
			ret += __builtin_popcount(eq_pairs(gv_word16(a, pos + (uint32_t)i) ^ rt_word16(t, o + i)));
		if (i < test_len) {
			const uint32_t mask = (1u << ((test_len - i) * 2)) - 1;
			ret += __builtin_popcount(eq_pairs(gv_word16(a, pos + (uint32_t)i) ^ rt_word16(t, o + i)) & mask);
		}
		return ret;
	}
	/* the literal loop (array end, reads past the text's end: NUL never matches) */
	int ret = 0;
	uint32_t bit = pos % 4 * 2;
	int8_t iv = (int8_t)a->values[byte];
	for (int i = 0; i < test_len; i++) {
		const int tt = (iv >> bit) & 3;
		const int k = o + i;
		const char c = (k >= 0 && k < t->len) ? t->text[k] : 0;
		switch (c) {
		case 'A': ret += tt == 0; break;
		case 'G': ret += tt == 1; break;
		case 'C': ret += tt == 2; break;
		case 0: break;
		default: ret += tt == 3;
		}
		bit += 2;
		if (bit == 8) {
			byte++;
			if (byte == a->values_bytes) return 0;
			iv = (int8_t)a->values[byte];
			bit = 0;
		}
	}
	return ret;
}

/* per-base equality of the read's characters from o with gvindex_get's characters from pos, for
 * len bases: bit i of m */
static void match_bits(const rtext *t, int o, const garray *a, uint32_t pos, int len, uint64_t *m)
{
	memset(m, 0, sizeof(uint64_t) * (size_t)((len + 63) / 64 + 1));
	if (len <= 0) return;
	const uint32_t rel = pos - a->start_base_offset;
	const int fast = pos >= a->start_base_offset && o >= 0 && o + len <= t->len &&
	                 (uint64_t)(rel >> 2) + (uint64_t)(len + 3) / 4 + 10 < a->values_bytes;
	if (fast) {
		for (int i = 0; i < len; i += 16) {
			uint32_t e = eq_pairs(gv_word16(a, pos + (uint32_t)i) ^ rt_word16(t, o + i));
			/* compress the 16 even bits to 16 bits */
			uint32_t x = e;
			x = (x | (x >> 1)) & 0x33333333u;
			x = (x | (x >> 2)) & 0x0f0f0f0fu;
			x = (x | (x >> 4)) & 0x00ff00ffu;
			x = (x | (x >> 8)) & 0x0000ffffu;
			/* a character other than A C G T never equals the array's base */
			const int k = o + i, w = k >> 6, s = k & 63;
			uint64_t od = t->odd[w] >> s;
			if (s) od |= t->odd[w + 1] << (64 - s);
			x &= ~(uint32_t)(od & 0xffff);
			const int n = len - i < 16 ? len - i : 16;
			if (n < 16) x &= (1u << n) - 1;
			m[i >> 6] |= (uint64_t)x << (i & 63);
		}
		return;
	}
	for (int i = 0; i < len; i++) {
		const int k = o + i;
		const char c = (k >= 0 && k < t->len) ? t->text[k] : 0;
		if (c == gv_char(a, pos + (uint32_t)i)) m[i >> 6] |= 1ull << (i & 63);
	}
}

static inline int mbit(const uint64_t *m, int i) { return (int)((m[i >> 6] >> (i & 63)) & 1); }

/* find_soft_clipping (core-junction.c:2820-2895) on the section's match bits */
#define SC_WIN 5
#define SC_ERR 1
static int soft_clip(const uint64_t *m, int test_len, int to_tail, int center)
{
	int base_in_window = 0, added, removed, search_start, matched = SC_WIN, last_matched = -1, delta;
	if (to_tail) {
		if (center < 0) search_start = 0;
		else if (center >= test_len) search_start = test_len - 1;
		else search_start = center - 1;
		delta = 1;
	} else {
		if (center < 0) search_start = 0;
		else if (center >= test_len) search_start = test_len - 1;
		else search_start = center + 1;
		delta = -1;
	}
	for (added = search_start; added >= 0 && added < test_len; added += delta) {
		const int am = mbit(m, added);
		matched += am;
		if (am) last_matched = added;
		base_in_window++;
		if (base_in_window > SC_WIN) {
			removed = added - delta * SC_WIN;
			matched -= mbit(m, removed);
		} else matched--;
		if (matched < SC_WIN - SC_ERR) {
			if (to_tail) return last_matched < 0 ? test_len - search_start : test_len - last_matched - 1;
			return last_matched >= 0 ? last_matched : search_start - 1;
		}
	}
	if (last_matched < 0) return test_len;
	if (to_tail) return test_len - last_matched - 1;
	return last_matched;
}

/* ------------------------------------------------------------------ explain_read */
typedef struct {
	int16_t start, end;        /* read_pos_start / read_pos_end */
	uint32_t abs;              /* abs_offset_for_start */
	int8_t jumped, to_large;   /* is_strand_jumped / is_connected_to_large_side */
	int32_t ev;                /* event_after_section (-1: NULL) */
} sec_t;

typedef struct {
	uint8_t tmp_n;
	sec_t tmp[MAX_EV_READ];
	sec_t back[MAX_ALN][MAX_EV_READ], front[MAX_ALN][MAX_EV_READ];
	int back_n[MAX_ALN], front_n[MAX_ALN], all_back, all_front;
	uint32_t total_tries;
	int best_matching, best_second_diff, second_best_matching, best_indel_penalty, tmp_total_matched, tmp_indel_penalty,
	    is_currently_tie, best_is_complex, best_support_as_simple, best_min_unsupport_as_simple, best_min_support_as_complex,
	    best_is_pure;
	int tmp_support_as_simple, tmp_min_unsupport, tmp_min_support_as_complex, tmp_is_pure;
	int full_read_len;
} xc_t;

/* realignment_result_t (core.h:372-391), the fields read after finalise_explain_CIGAR */
typedef struct {
	int rec;                          /* the mapping record (index into the chunk's records) */
	uint32_t first_base_position;
	char cigar[CIGAR_LEN];
	int32_t support[MAX_EV_READ];     /* supporting_chromosome_events (-1 ends the list) */
	int16_t flank_l[MAX_EV_READ], flank_r[MAX_EV_READ];
	int16_t final_mismatched, final_matched, realign_flags, chromosomal_length, mapq_adjustment;
	int32_t known_junction_supp, final_penalty;
} realign_t;

typedef struct {
	const svg_realign *ra;
	const garray *vi;                 /* the record's value index (locate_current_value_index) */
	const rtext *t;
	xc_t x;
	uint64_t mbits[MAXRL / 64 + 4];
} wk_t;

static void sec_clear(sec_t *s, int n)
{
	memset(s, 0, sizeof(sec_t) * (size_t)n);
	for (int i = 0; i < n; i++) s[i].ev = -1;
}

/* new_explain_try_replace, core-junction.c:308-447 */
static void try_replace(xc_t *x, int remainder_len, int to_back)
{
	int is_better = 0, is_same = 0;
	if (x->best_matching - x->best_indel_penalty < x->tmp_total_matched - x->tmp_indel_penalty) {
		is_better = 1;
		x->best_is_complex = x->tmp_n;
		x->is_currently_tie = 0;
		x->best_support_as_simple = x->tmp_support_as_simple;
		x->best_min_unsupport_as_simple = x->tmp_min_unsupport;
		x->best_min_support_as_complex = x->tmp_min_support_as_complex;
		x->best_is_pure = x->tmp_is_pure;
		x->second_best_matching = imax(x->second_best_matching, x->best_matching);
		x->best_matching = x->tmp_total_matched;
		x->best_indel_penalty = x->tmp_indel_penalty;
	} else if (x->best_matching - x->best_indel_penalty == x->tmp_total_matched - x->tmp_indel_penalty) {
		x->best_is_complex += x->tmp_n;
		x->second_best_matching = x->best_matching;
		x->best_indel_penalty = x->tmp_indel_penalty;
		if (x->best_is_complex > 1) {
			if (x->tmp_n == 0) {
				if (x->tmp_min_unsupport > x->best_min_support_as_complex) {
					is_better = 1;
					x->best_min_support_as_complex = x->tmp_min_unsupport;
					x->best_is_pure = x->tmp_is_pure;
					x->is_currently_tie = 0;
				} else if (x->tmp_min_unsupport == x->best_min_support_as_complex) {
					x->is_currently_tie = 1;
					is_same = 1;
				}
			} else {
				if (x->tmp_min_support_as_complex > x->best_min_support_as_complex) {
					is_better = 1;
					x->best_min_support_as_complex = x->tmp_min_support_as_complex;
					x->best_is_pure = x->tmp_is_pure;
					x->is_currently_tie = 0;
				} else if (x->tmp_min_support_as_complex == x->best_min_support_as_complex) {
					x->is_currently_tie = 1;
					is_same = 1;
				}
			}
		} else if (x->best_is_pure) {
			/* the last best is one-gapped and the current one ungapped */
			if (x->best_min_unsupport_as_simple >= x->best_support_as_simple + 2) {
				is_better = 1;
				x->best_min_support_as_complex = x->best_min_unsupport_as_simple;
				x->best_is_pure = x->tmp_is_pure;
				x->is_currently_tie = 0;
			}
		}
	} else return;

	if (is_better || is_same) {
		if (to_back) x->tmp[x->tmp_n].start = 0;
		else {
			x->tmp[x->tmp_n].end = (int16_t)(x->tmp[x->tmp_n].start + remainder_len);
			x->tmp[x->tmp_n].ev = -1;
		}
	}
	if (is_better) {
		if (to_back) {
			x->all_back = 1;
			x->back_n[0] = x->tmp_n + 1;
			memcpy(x->back[0], x->tmp, sizeof(sec_t) * (size_t)(x->tmp_n + 1));
		} else {
			x->all_front = 1;
			x->front_n[0] = x->tmp_n + 1;
			memcpy(x->front[0], x->tmp, sizeof(sec_t) * (size_t)(x->tmp_n + 1));
		}
	} else if (is_same) {
		if (to_back && x->all_back < MAX_ALN) {
			x->back_n[x->all_back] = x->tmp_n + 1;
			memcpy(x->back[x->all_back], x->tmp, sizeof(sec_t) * (size_t)(x->tmp_n + 1));
			x->all_back++;
		} else if (!to_back && x->all_front < MAX_ALN) {
			x->front_n[x->all_front] = x->tmp_n + 1;
			memcpy(x->front[x->all_front], x->tmp, sizeof(sec_t) * (size_t)(x->tmp_n + 1));
			x->all_front++;
		}
	}
}

/* search_events_to_back, core-junction.c:588-746 (no fusion / long-deletion detection: no
 * strand jumps).  tail_abs: the first unwanted base after the section; tail_pos: the first
 * unwanted read base (the read text from its start). */
static void search_back(wk_t *W, uint32_t tail_abs, int16_t tail_pos, int16_t sofar, int suggested, int no_jump)
{
	const svg_realign *ra = W->ra;
	const svg_realign_params *p = &ra->p;
	xc_t *x = &W->x;
	if (events_in_range(ra->bm_large, tail_abs - (uint32_t)tail_pos, tail_pos)) {
		int move_start = tail_pos - (no_jump ? 0 : p->realignment_minimum_variant_distance);
		if (suggested) move_start = tail_pos - suggested + 1;
		if (MAX_EV_READ - 1 > x->tmp_n)
			for (int16_t t = (int16_t)move_start; t >= 0; t--) {
				uint32_t ids[SITE_MAX];
				const uint32_t potential = tail_abs - (uint32_t)(tail_pos - t);
				const int n = search_side(ra, potential, 1, ids);
				if (!n) continue;
				const uint32_t chro_begin = tail_abs - (uint32_t)(tail_pos - t);
				const int matched = match_chro(W->t, t, W->vi, chro_begin, tail_pos - t);
				if (x->total_tries < TOTAL_TRIES && tail_pos > t &&
				    (matched * 10000 / (tail_pos - t) > 9000 - 2000 || p->maximise_sensitivity_indel))
					for (int k = 0; k < n; k++) {
						const svg_event *e = &ra->ev[ids[k]];
						int new_tail_pos = t;
						if (e->event_type == EV_INDEL) new_tail_pos += imin(0, e->indel_length);
						const uint32_t new_tail_abs = e->small_side + 1;
						new_tail_pos -= e->indel_at_junction;
						if (new_tail_pos > 0) {
							x->tmp[x->tmp_n].start = t;
							x->tmp[x->tmp_n + 1].ev = (int32_t)ids[k];
							x->tmp[x->tmp_n + 1].to_large = potential == e->small_side;
							x->tmp[x->tmp_n + 1].end = (int16_t)(t + imin(0, e->indel_length) - e->indel_at_junction);
							x->tmp[x->tmp_n + 1].abs = new_tail_abs;
							const int cur_sup_complex = x->tmp_min_support_as_complex, cur_sup_simple = x->tmp_support_as_simple,
							          cur_pure = x->tmp_is_pure;
							x->tmp_support_as_simple = e->supporting_reads;
							x->tmp_min_support_as_complex = imin((e->is_donor_found_or_annotation & 64) ? 0x7fffffff : e->supporting_reads,
							                                     x->tmp_min_support_as_complex);
							x->tmp_min_unsupport = imin(e->anti_supporting_reads, x->tmp_min_unsupport);
							x->tmp_is_pure = x->tmp_is_pure && e->is_donor_found_or_annotation;
							x->tmp_indel_penalty += e->event_type == EV_INDEL;
							x->tmp[x->tmp_n + 1].jumped = 0;
							x->tmp_n++;
							x->total_tries++;
							search_back(W, new_tail_abs, (int16_t)new_tail_pos, (int16_t)(sofar + matched), e->connected_previous_event_distance, 0);
							x->tmp_n--;
							x->tmp_indel_penalty -= e->event_type == EV_INDEL;
							x->tmp_min_support_as_complex = cur_sup_complex;
							x->tmp_support_as_simple = cur_sup_simple;
							x->tmp_is_pure = cur_pure;
							/* (tmp_min_unsupport is not restored, core-junction.c:290) */
						}
					}
				if (p->limited_tree_scan && x->full_read_len <= LONG_READ) break;
			}
	}
	const int whole = match_chro(W->t, 0, W->vi, tail_abs - (uint32_t)tail_pos, tail_pos);
	x->tmp_total_matched = whole + sofar;
	try_replace(x, 0, 1);
}

/* search_events_to_front, core-junction.c:125-306.  toff: the read offset of the section's
 * first base; head_abs: its position; remainder: bases to the read's end. */
static void search_front(wk_t *W, int toff, uint32_t head_abs, int16_t remainder, int16_t sofar, int suggested, int no_jump)
{
	const svg_realign *ra = W->ra;
	const svg_realign_params *p = &ra->p;
	xc_t *x = &W->x;
	if (events_in_range(ra->bm_small, head_abs, remainder)) {
		int move_start = no_jump ? 0 : p->realignment_minimum_variant_distance;
		if (suggested) move_start = suggested - 1;
		if (MAX_EV_READ - 1 > x->tmp_n)
			for (int16_t t = (int16_t)move_start; t <= remainder; t++) {
				uint32_t ids[SITE_MAX];
				const uint32_t potential = head_abs + (uint32_t)t - 1;
				const int n = search_side(ra, potential, 0, ids);
				if (!n) continue;
				const int matched = match_chro(W->t, toff, W->vi, head_abs, t);
				if (x->total_tries < TOTAL_TRIES && t > 0 && (matched * 10000 / t > 9000 - 2000 || p->maximise_sensitivity_indel))
					for (int k = 0; k < n; k++) {
						const svg_event *e = &ra->ev[ids[k]];
						const uint32_t new_head = e->large_side;
						const int16_t new_rem = (int16_t)(remainder - t + imin(0, e->indel_length) - e->indel_at_junction);
						if (new_rem > 0) {
							x->tmp[x->tmp_n].end = (int16_t)(x->tmp[x->tmp_n].start + t);
							x->tmp[x->tmp_n].ev = (int32_t)ids[k];
							x->tmp[x->tmp_n].to_large = potential == e->large_side;
							x->tmp[x->tmp_n + 1].start = (int16_t)(t - imin(0, e->indel_length) + e->indel_at_junction);
							x->tmp[x->tmp_n + 1].abs = new_head;
							const int cur_sup_complex = x->tmp_min_support_as_complex, cur_sup_simple = x->tmp_support_as_simple,
							          cur_pure = x->tmp_is_pure;
							x->tmp_support_as_simple = e->supporting_reads;
							x->tmp_min_support_as_complex = imin((e->is_donor_found_or_annotation & 64) ? 0x7fffffff : e->supporting_reads,
							                                     x->tmp_min_support_as_complex);
							x->tmp_min_unsupport = imin(e->anti_supporting_reads, x->tmp_min_unsupport);
							x->tmp_is_pure = x->tmp_is_pure && e->is_donor_found_or_annotation;
							x->tmp_indel_penalty += e->event_type == EV_INDEL;
							x->tmp[x->tmp_n + 1].jumped = 0;
							x->tmp_n++;
							x->total_tries++;
							search_front(W, toff + e->indel_at_junction + t - imin(0, e->indel_length), new_head, new_rem,
							             (int16_t)(sofar + matched), e->connected_next_event_distance, 0);
							x->tmp_n--;
							x->tmp_indel_penalty -= e->event_type == EV_INDEL;
							x->tmp_min_support_as_complex = cur_sup_complex;
							x->tmp_support_as_simple = cur_sup_simple;
							x->tmp_is_pure = cur_pure;
						}
					}
				if (p->limited_tree_scan && x->full_read_len <= LONG_READ) break;
			}
	}
	const int whole = match_chro(W->t, toff, W->vi, head_abs, remainder);
	x->tmp_total_matched = whole + sofar;
	try_replace(x, remainder, 0);
}

/* final_CIGAR_quality, core-junction.c:2899-3156 (no strand-jumped sections): soft clipping of
 * the first / last M section, the mismatches, the clipped CIGAR.  Returns nothing the caller
 * uses beyond the out-parameters (the quality score is not computed, see the file header). */
static void final_cigar_quality(wk_t *W, int read_len, char *cigar, uint32_t head_abs, int *mismatched, int covered_start,
                                int covered_end, int *matched_bases, int *chromosomal_length)
{
	const svg_realign_params *p = &W->ra->p;
	const garray *a = W->vi;
	int cur = 0, read_cursor = 0, rebuilt = 0, total_ins = 0, all_mm = 0, is_first_m = 1, wrong = 0;
	int head_clip = -1, tail_clip = -1;
	uint32_t abs = head_abs, tmp = 0;
	for (;;) {
		const char nch = cigar[cur++];
		if (!nch) break;
		if (is_digit(nch)) { tmp = tmp * 10 + (uint32_t)(nch - '0'); continue; }
		if (tmp == 0) wrong = 1;
		if (wrong) break;
		if (nch == 'M' || nch == 'S') {
			const int is_last_m = cigar[cur] == 0, len = (int)tmp;
			int has_head = 0, has_tail = 0;
			match_bits(W->t, read_cursor, a, abs, len, W->mbits);
			if (is_first_m && p->show_soft_clipping) {
				head_clip = soft_clip(W->mbits, len, 0, covered_start - read_cursor);
				if (head_clip == len) head_clip = 0;
				else has_head = 1;
			}
			if (is_last_m && p->show_soft_clipping) {
				tail_clip = soft_clip(W->mbits, len, 1, covered_end - read_cursor);
				if (tail_clip == len) tail_clip = 0;
				else has_tail = 1;
			}
			if (is_last_m && is_first_m && tail_clip + head_clip >= len - 1) { head_clip = 0; tail_clip = 0; }
			const int mm_start = has_head ? head_clip : 0, mm_end = has_tail ? tail_clip : 0;
			/* match_base_quality (gene-algorithms.c:2012-2080): nothing counted outside the array */
			if (!(abs < a->start_base_offset || abs + (uint32_t)len >= a->start_base_offset + a->length))
				for (int i = mm_start; i < len - mm_end; i++) all_mm += !mbit(W->mbits, i);
			rebuilt += len;
			is_first_m = 0;
			read_cursor += len;
			abs += tmp;
		} else if (nch == 'I') {
			rebuilt += (int)tmp;
			read_cursor += (int)tmp;
			total_ins += (int)tmp;
		} else if (nch == 'D') abs += tmp;
		else if (nch == 'N' || nch == 'n') abs += tmp;
		else if (nch == 'B' || nch == 'b') abs -= tmp;
		if (read_cursor > MAXRL) wrong = 1;
		tmp = 0;
	}
	int non_clipped = read_len - imax(0, tail_clip) - imax(0, head_clip);
	if (wrong || rebuilt != read_len || non_clipped < p->min_mapped_fraction) {
		*mismatched = 99999;
		snprintf(cigar, 11, "%dM", read_len);
	} else if (head_clip > 0 || tail_clip > 0) {
		char nc[120], piece[30], tiny[12];
		int first = 1;
		nc[0] = 0;
		cur = 0;
		for (;;) {
			const char nch = cigar[cur++];
			if (!nch) break;
			if (is_digit(nch)) { tmp = tmp * 10 + (uint32_t)(nch - '0'); continue; }
			piece[0] = 0;
			if (nch == 'M') {
				const int is_last_m = cigar[cur] == 0;
				if (first && head_clip > 0) {
					tmp -= (uint32_t)head_clip;
					snprintf(tiny, 11, "%dS", head_clip);
					strcat(piece, tiny);
				}
				if (is_last_m && tail_clip > 0) tmp -= (uint32_t)tail_clip;
				snprintf(tiny, 11, "%dM", (int)tmp);
				strcat(piece, tiny);
				if (is_last_m && tail_clip > 0) {
					snprintf(tiny, 11, "%dS", tail_clip);
					strcat(piece, tiny);
				}
				first = 0;
			} else snprintf(piece, 11, "%u%c", tmp, nch);
			strcat(nc, piece);
			tmp = 0;
		}
		strcpy(cigar, nc);
	}
	if (*mismatched != 99999) *mismatched = all_mm;
	*matched_bases = non_clipped - all_mm - total_ins;
	*chromosomal_length = (int)(abs - head_abs) + total_ins;
}

/* finalise_explain_CIGAR, core-junction.c:3159-3449 (no fusions); the accepted alignments go to
 * out[0..] (at most MAX_ALN) */
static int finalise_cigar(wk_t *W, svg_mapping_result *result, int rec_index, realign_t *out)
{
	const svg_realign *ra = W->ra;
	const svg_realign_params *p = &ra->p;
	xc_t *x = &W->x;
	int is_junction_read = 0, is_cigar_overflow = 0, fusions_in_read = 0, final_n = 0;
	char tmp_cigar[120];
	int32_t to_be_supported[20];
	int16_t flank_l[20], flank_r[20];
	int to_be_supported_count = 0;
	result->result_flags &= (int16_t)~F_FULLY;
	result->result_flags &= (int16_t)~F_PAIRED_END;
	for (int b = 0; b < x->all_back; b++) {
		if (x->back_n[b] > MAX_EV_READ) return 0;
		for (int k = 0; k < x->back_n[b] / 2; k++) {
			const sec_t t = x->back[b][k];
			x->back[b][k] = x->back[b][x->back_n[b] - k - 1];
			x->back[b][x->back_n[b] - k - 1] = t;
		}
	}
	for (int b = 0; b < x->all_back; b++) {
		if (final_n >= MAX_ALN) break;
		for (int k = 0; k < x->back_n[b]; k++) {
			const int section_length = x->back[b][k].end - x->back[b][k].start;
			x->back[b][k].abs = x->back[b][k].abs - (uint32_t)section_length;
		}
		for (int f = 0; f < x->all_front; f++) {
			if (final_n >= MAX_ALN) break;
			to_be_supported_count = 0;
			tmp_cigar[0] = 0;
			int known_junction_supp = 0;
			const int nsec = x->back_n[b] + x->front_n[f] - 1;
			for (int k = 0; k < nsec; k++) {
				char piece[25];
				const sec_t *cs, *ns = NULL;
				if (k >= x->back_n[b] - 1) {
					cs = &x->front[f][k - x->back_n[b] + 1];
					if (k - x->back_n[b] + 2 < x->front_n[f]) ns = &x->front[f][k - x->back_n[b] + 2];
				} else {
					cs = &x->back[b][k];
					if (k + 1 < x->back_n[b]) ns = &x->back[b][k + 1];
				}
				(void)ns;
				const int rps = k == x->back_n[b] - 1 ? x->back[b][k].start : cs->start;
				const int rpe = cs->end;
				snprintf(piece, 11, "%dM", rpe - rps);
				flank_l[k] = (int16_t)(rpe - rps);
				if (k > 0) flank_r[k - 1] = (int16_t)(rpe - rps);
				if (cs->ev >= 0) {
					const svg_event *e = &ra->ev[cs->ev];
					if (e->event_type == EV_INDEL)
						snprintf(piece + strlen(piece), 11, "%d%c", abs(e->indel_length), e->indel_length > 0 ? 'D' : 'I');
					else if (e->event_type == EV_JUNCTION || e->event_type == EV_FUSION) {
						const int delta_one = (cs->jumped + cs->to_large == 1) ? 1 : -1;
						char jump_mode = cs->to_large ? 'B' : 'N';
						long long movement = e->large_side;
						movement -= (long long)e->small_side - delta_one;
						if (jump_mode == 'B' && movement < 0) { movement = -movement; jump_mode = 'N'; }
						else if (jump_mode == 'N' && movement < 0) { movement = -movement; jump_mode = 'B'; }
						fusions_in_read += e->event_type == EV_FUSION;
						snprintf(piece + strlen(piece), 11, "%u%c", (unsigned)(int)movement, jump_mode);
						if (e->indel_at_junction) snprintf(piece + strlen(piece), 11, "%dI", e->indel_at_junction);
						is_junction_read++;
						if (e->is_donor_found_or_annotation & 64) known_junction_supp++;
					}
					to_be_supported[to_be_supported_count++] = cs->ev;
				}
				strcat(tmp_cigar, piece);
				if (strlen(tmp_cigar) > CIGAR_LEN - 14) {
					is_cigar_overflow = 1;
					break;
				}
			}
			int mismatch_bases = 0;
			if (is_cigar_overflow) snprintf(tmp_cigar, 11, "%dM", x->full_read_len);
			const uint32_t final_position = x->back[b][0].abs;
			int is_exonic_ok = 1;
			if (p->minimum_exonic_subread_fraction > 0.0000001f && !is_junction_read && result->used_subreads_in_vote > 0) {
				const int min_subreads = (int)(p->minimum_exonic_subread_fraction * result->used_subreads_in_vote);
				if (result->selected_votes < min_subreads) is_exonic_ok = 0;
			}
			int applied_mismatch = 0, final_match = 0, chromosomal_length = 0;
			if (is_exonic_ok) {
				final_cigar_quality(W, x->full_read_len, tmp_cigar, final_position, &mismatch_bases, result->confident_coverage_start,
				                    result->confident_coverage_end, &final_match, &chromosomal_length);
				applied_mismatch = is_junction_read ? p->max_mismatch_junction : p->max_mismatch_exonic;
				if (x->full_read_len > LONG_READ)
					applied_mismatch = ((((x->full_read_len + 1) << 16) / 100) * applied_mismatch) >> 16;
			}
			if (mismatch_bases <= applied_mismatch && is_exonic_ok && fusions_in_read < 2) {
				realign_t *rr = &out[final_n++];
				rr->rec = rec_index;
				rr->realign_flags = result->result_flags;
				rr->chromosomal_length = (int16_t)chromosomal_length;
				rr->known_junction_supp = known_junction_supp;
				rr->final_penalty = x->best_indel_penalty;
				rr->realign_flags &= (int16_t)~F_TOO_MANY;
				strcpy(rr->cigar, tmp_cigar);
				int is_rna_from_positive = -1;
				for (int k = 0; k < to_be_supported_count; k++) {
					if (k >= MAX_EV_READ) break;
					const svg_event *e = &ra->ev[to_be_supported[k]];
					if (e->event_type != EV_INDEL && is_junction_read)
						if (e->event_type == EV_JUNCTION && e->is_donor_found_or_annotation && is_rna_from_positive == -1)
							is_rna_from_positive = !e->is_negative_strand;
					rr->support[k] = to_be_supported[k];
					rr->flank_l[k] = flank_l[k];
					rr->flank_r[k] = flank_r[k];
				}
				if (to_be_supported_count < MAX_EV_READ) rr->support[to_be_supported_count] = -1;
				result->result_flags |= F_FULLY;
				result->read_length = (int16_t)x->full_read_len;
				if (is_rna_from_positive == -1) {
					rr->realign_flags |= F_NOTFOUND;
					rr->realign_flags &= (int16_t)~F_GT_AG;
				} else {
					rr->realign_flags &= (int16_t)~(F_NOTFOUND | F_GT_AG);
					if (is_rna_from_positive) rr->realign_flags |= F_GT_AG;
				}
				rr->first_base_position = final_position;
				rr->final_mismatched = (int16_t)mismatch_bases;
				rr->final_matched = (int16_t)(uint16_t)final_match;
				rr->mapq_adjustment = 0;
			}
		}
	}
	return final_n;
}

/* explain_read, core-junction.c:2617-2777 */
static int explain_read(wk_t *W, svg_mapping_result *result, int rec_index, int read_len, realign_t *out)
{
	xc_t *x = &W->x;
	memset(x, 0, sizeof *x);
	sec_clear(x->tmp, MAX_EV_READ);
	x->full_read_len = read_len;
	const unsigned short back_tail = (unsigned short)imin(read_len, result->confident_coverage_end);
	const uint32_t back_tail_pos = result->selected_position + back_tail + (uint32_t)(int)result->indels_in_confident_coverage;
	x->tmp[0].end = (int16_t)back_tail;
	x->tmp[0].abs = back_tail_pos;
	x->all_back = 0;
	x->tmp_n = 0;
	x->best_indel_penalty = 0;
	x->best_matching = -9999;
	x->second_best_matching = -9999;
	x->tmp_indel_penalty = 0;
	x->tmp_total_matched = 0;
	x->is_currently_tie = 0;
	x->best_is_complex = 0;
	x->best_support_as_simple = 0;
	x->best_min_unsupport_as_simple = 0;
	x->tmp_support_as_simple = 0;
	x->tmp_min_support_as_complex = 999999;
	x->tmp_min_unsupport = 999999;
	x->tmp_is_pure = 1;
	x->best_is_pure = 0;
	const unsigned short front_read_start = back_tail > 8 ? back_tail - 8 : 0;
	const uint32_t front_start_pos = back_tail_pos > 8 ? back_tail_pos - 8 : 0;
	search_back(W, back_tail_pos, (int16_t)back_tail, 0, 0, 1);
	const int back_penalty = x->best_indel_penalty;
	const int back_diff = -9999;
	x->all_front = 0;
	x->tmp_n = 0;
	x->best_indel_penalty = 0;
	x->best_matching = -9999;
	x->second_best_matching = -9999;
	x->tmp_total_matched = 0;
	x->tmp_indel_penalty = 0;
	x->is_currently_tie = 0;
	x->best_is_complex = 0;
	x->best_support_as_simple = 0;
	x->best_min_unsupport_as_simple = 0;
	x->tmp_support_as_simple = 0;
	x->tmp_min_support_as_complex = 999999;
	x->tmp_min_unsupport = 999999;
	x->tmp_is_pure = 1;
	x->best_is_pure = 0;
	sec_clear(x->tmp, MAX_EV_READ);
	x->tmp[0].start = (int16_t)front_read_start;
	x->tmp[0].abs = front_start_pos;
	const int16_t search_remain = (int16_t)(read_len - front_read_start);
	search_front(W, front_read_start, front_start_pos, search_remain, 0, 0, 1);
	x->best_indel_penalty += back_penalty;
	x->best_second_diff = x->best_matching - x->second_best_matching + back_diff;
	return finalise_cigar(W, result, rec_index, out);
}

/* ------------------------------------------------------------------ SAM fields */
/* locate_gene_position_max, gene-algorithms.c:441-511 (head / tail cut pointers NULL when the
 * caller passes NULL): contig index in *chr (-1 = NULL name) */
static int locate_max(const svg_genome_arrays *g, uint32_t linear, int *chr, int *pos, int *head_cut, int *tail_cut, int rl)
{
	int n = 0;
	*chr = -1;
	*pos = -1;
	int lo = 0, hi = (int)g->n_chr;
	for (;;) {
		if (hi <= lo + 1) { n = imax(lo - 2, 0); break; }
		const int mid = (lo + hi) / 2;
		if (g->chr_end[mid] > linear) hi = mid;
		else lo = mid + 1;
	}
	for (; n < (int)g->n_chr; n++) {
		if (g->chr_end[n] > linear) {
			*pos = n == 0 ? (int)linear : (int)(linear - g->chr_end[n - 1]);
			if (!tail_cut) {
				if ((uint32_t)rl + linear > g->chr_end[n] + 15u - (uint32_t)g->padding) return 1;
			} else {
				const uint32_t posn1 = n > 0 ? g->chr_end[n - 1] : 0;
				long long tct = (long long)(linear + (uint32_t)rl - posn1 - (uint32_t)g->padding);
				if (tct < rl) tct = rl;
				const long long chro_leng = (long long)(g->chr_end[n] - posn1 - 2 * (uint32_t)g->padding + 16);
				tct -= chro_leng;
				if (tct >= rl) return 1;
				if (tct < 0) tct = 0;
				*tail_cut = (int)tct;
			}
			if (*pos < g->padding) {
				if (!head_cut || *pos + rl <= g->padding) return 1;
				*head_cut = g->padding - *pos;
				*pos = g->padding;
			}
			*pos -= g->padding;
			*chr = n;
			return 0;
		}
	}
	return -1;
}

static int soft_clip_len(const char *cigar)   /* get_soft_clipping_length, core.c:1232-1246 */
{
	int tmp = 0;
	for (int i = 0; cigar[i] > 0; i++) {
		if (is_digit(cigar[i])) tmp = tmp * 10 + (cigar[i] - '0');
		else return cigar[i] == 'S' ? tmp : 0;
	}
	return 0;
}

/* add_head_tail_cut_softclipping, core.c:1367-1421 */
static int add_head_tail_cut(char *cigar, int rlen, int head_cut, int tail_cut)
{
	char added[CIGAR_LEN];
	int cur = 0, ap = 0, read_cursor = 0, next_read_cursor = 0, tmpi = 0, nch, has_m = 0;
	added[0] = 0;
	for (;;) {
		nch = cigar[cur++];
		if (nch == 0) break;
		if (is_digit(nch)) { tmpi = 10 * tmpi + (nch - '0'); continue; }
		if (nch == 'M' || nch == 'S' || nch == 'I') next_read_cursor = read_cursor + tmpi;
		int head_s = 0, tail_s = 0, rem = tmpi, skip = 0;
		if (next_read_cursor <= head_cut) skip = 1;
		if (read_cursor >= rlen - tail_cut) skip = 1;
		if (!skip) {
			if (nch != 'S') {
				if (read_cursor <= head_cut) head_s = head_cut;
				if (next_read_cursor >= rlen - tail_cut) tail_s = tail_cut;
				rem = tmpi;
				if (head_s) rem -= head_s - read_cursor;
				if (tail_s) rem -= next_read_cursor - (rlen - tail_s);
			}
			if ((head_s > 0 || tail_s > 0) && nch != 'M') return 0;
			if (head_s > 0) ap += snprintf(added + ap, (size_t)(CIGAR_LEN - ap), "%dS", head_s);
			if (rem > 0) {
				ap += snprintf(added + ap, (size_t)(CIGAR_LEN - ap), "%d%c", rem, nch);
				if (nch == 'M') has_m = 1;
			}
			if (tail_s > 0) ap += snprintf(added + ap, (size_t)(CIGAR_LEN - ap), "%dS", tail_s);
		}
		read_cursor = next_read_cursor;
		tmpi = 0;
	}
	strcpy(cigar, added);
	return has_m;
}

/* subread_output_tmp_t (core.c:1249-1284), the fields write_single_fragment reads */
typedef struct {
	int ok, chr, strand, mapq, soft;
	int offset;
	uint32_t linear;
	char cigar[CIGAR_LEN + 8];
	char info[64];                   /* additional_information: "\tXS:A:+" */
	const realign_t *res;
} outrec;

/* convert_read_to_tmp, core.c:1424-1535 */
static int convert_rec(const svg_realign *ra, const realign_t *res, const svg_mapping_result *mr, int read_len, outrec *r)
{
	const svg_realign_params *p = &ra->p;
	r->res = res;
	r->info[0] = 0;
	int ok = (mr->result_flags & F_FULLY) > 0;
	if (ok) {
		snprintf(r->cigar, sizeof r->cigar, "%s", res->cigar);
		r->linear = res->first_base_position;
		r->mapq = 40;
		if (res->realign_flags & F_BREAKEVEN) r->mapq = 0;
		else r->mapq /= res->mapq_adjustment;
		r->strand = (mr->result_flags & F_NEG) ? 1 : 0;
		r->soft = soft_clip_len(r->cigar);
	}
	if (ok) {
		int head_cut = 0, tail_cut = 0;
		if (locate_max(ra->g, r->linear + (uint32_t)r->soft, &r->chr, &r->offset, &head_cut, &tail_cut, res->chromosomal_length - r->soft))
			ok = 0;
		else {
			int added = 1;
			if (head_cut || tail_cut) added = add_head_tail_cut(r->cigar, read_len, head_cut, tail_cut);
			if (added) r->offset++;
			else ok = 0;
		}
		if (p->do_breakpoint_detection && !(res->realign_flags & F_NOTFOUND))
			snprintf(r->info, sizeof r->info, "\tXS:A:%c", (res->realign_flags & F_GT_AG) ? '+' : '-');
	}
	r->ok = ok;
	return ok;
}

/* calc_tlen, core.c:1718-1789 */
static int calc_tlen(const outrec *r1, const outrec *r2, int len1, int len2)
{
	int ret = -1;
	const uint32_t h1 = (uint32_t)r1->offset, h2 = (uint32_t)r2->offset;
	if (h1 == h2) return imax(len1, len2);
	const int r2_smaller = h2 < h1;
	const outrec *sm = r2_smaller ? r2 : r1;
	const uint32_t small_head = r2_smaller ? h2 : h1, large_head = r2_smaller ? h1 : h2;
	const int len_larger = r2_smaller ? len1 : len2, len_smaller = r2_smaller ? len2 : len1;
	uint32_t tmpi = 0, chro_cursor = small_head, section_end = 0, read_cursor = 0;
	for (int c = 0;; c++) {
		const int nch = sm->cigar[c], nch2 = sm->cigar[c + 1];
		if (nch <= 0) break;
		if (is_digit(nch)) { tmpi = tmpi * 10 + (uint32_t)(nch - '0'); continue; }
		if (nch == 'M' || nch == 'S') { chro_cursor += tmpi; read_cursor += tmpi; section_end = chro_cursor; }
		if (nch == 'N' || nch == 'B' || nch == 'b' || nch == 'n' || nch == 'I' || nch == 'D' || nch2 == 0) {
			if (nch == 'N' || nch == 'D') chro_cursor += tmpi;
			if (section_end >= large_head) {
				ret = (int)(read_cursor + large_head - section_end + (uint32_t)len_larger);
				break;
			}
		}
		if (nch == 'I') read_cursor += tmpi;
		if (nch == 'B' || nch == 'b' || nch == 'n') break;
		tmpi = 0;
	}
	if (ret < 0) ret = (int)(large_head - section_end + (uint32_t)len_larger + (uint32_t)len_smaller);
	return ret;
}

typedef struct {
	svg_realign_stats st;
	uint32_t *ev_count;              /* final_counted_reads added, per event */
	int16_t *ev_fl, *ev_fr;          /* flanking maxima, per event (INT16_MIN: none) */
} tally_t;

/* calc_flags, core.c:1635-1715 */
static int calc_flags(const svg_realign *ra, tally_t *T, const outrec *rec1, const outrec *rec2, int is_second, int loc, int tlen,
                      int this_ok, int mate_ok)
{
	const svg_realign_params *p = &ra->p;
	int ret, tlen_wrong = 0;
	if (p->paired) {
		ret = S_PAIRED | (is_second ? S_SECOND : S_FIRST);
		const outrec *th = is_second ? rec2 : rec1, *ma = is_second ? rec1 : rec2;
		if (!this_ok) ret |= S_UNMAPPED;
		else if (th->strand + is_second == 1) ret |= S_REVERSE;
		if (!mate_ok) ret |= S_MATE_UNMAP;
		else if (ma->strand + is_second != 1) ret |= S_MATE_REV;
		if (rec1 && rec2) {
			int pem = 0;
			if (rec1->chr == rec2->chr && tlen >= p->min_pair_distance && tlen <= p->max_pair_distance && th->strand == ma->strand) {
				if (p->is_first_read_reversed && !p->is_second_read_reversed) {
					if (th->strand == 0) {
						if ((is_second + (ma->offset > th->offset) == 1) || ma->offset == th->offset) pem = 1;
						else tlen_wrong = 1;
					}
				} else if (th->strand) {
					if ((is_second + (ma->offset < th->offset) == 1) || ma->offset == th->offset) pem = 1;
					else tlen_wrong = 1;
				} else {
					if ((is_second + (ma->offset > th->offset) == 1) || ma->offset == th->offset) pem = 1;
					else tlen_wrong = 1;
				}
			}
			if (pem) ret |= S_PROPER;
			else if (is_second) {
				if (rec1->chr != rec2->chr) T->st.not_properly_pairs_different_chro++;
				else if (th->strand != ma->strand) T->st.not_properly_different_strands++;
				else if (tlen < p->min_pair_distance || tlen > p->max_pair_distance) T->st.not_properly_pairs_TLEN_wrong++;
				else if (tlen_wrong) T->st.not_properly_pairs_wrong_arrangement++;
			}
		}
	} else {
		ret = 0;
		if (!this_ok) ret |= S_UNMAPPED;
		else if (rec1->strand) ret |= S_REVERSE;
	}
	if (loc > 0)
		if ((rec1 && !is_second) || (rec2 && is_second)) ret |= S_SECONDARY;
	return ret;
}

/* __converting_char_table of reverse_read (input-files.c:1111) */
static char revc_tab[256];
static pthread_once_t revc_once = PTHREAD_ONCE_INIT;
static void revc_init(void)
{
	for (int i = 0; i < 256; i++) { code_tab[i] = 3; odd_tab[i] = 1; }
	code_tab['A'] = 0; code_tab['G'] = 1; code_tab['C'] = 2;
	odd_tab['A'] = odd_tab['C'] = odd_tab['G'] = odd_tab['T'] = 0;
	/* the table maps A C G T U to T G C A A and every other character below 128 (lower case
	 * too) to N; 128 + 'A' etc. hold the same letters */
	for (int i = 0; i < 256; i++) revc_tab[i] = 'N';
	const char *from = "ACGTU", *to = "TGCAA";
	for (int k = 0; k < 5; k++) {
		revc_tab[(unsigned char)from[k]] = to[k];
		revc_tab[(unsigned char)from[k] + 128] = to[k];
	}
}

/* reverse_read (input-files.c:1113-1190, base space) into dst */
static void revcomp(char *dst, const char *src, int len)
{
	for (int i = 0; i < len; i++) dst[i] = revc_tab[(unsigned char)src[len - 1 - i]];
	dst[len] = 0;
}

static void revstr(char *dst, const char *src, int len)   /* reverse_quality, input-files.c:1192 */
{
	for (int i = 0; i < len; i++) dst[i] = src[len - 1 - i];
	dst[len] = 0;
}

/* calc_edit_dist, core.c:1325-1348 */
static int edit_dist(const char *cigar, int all_mm)
{
	unsigned tmpi = 0;
	for (int c = 0; cigar[c]; c++) {
		const char nch = cigar[c];
		if (is_digit(nch)) tmpi = tmpi * 10 + (unsigned)(nch - '0');
		else {
			if (nch == 'I' || nch == 'D') all_mm += (int)tmpi;
			tmpi = 0;
		}
	}
	return all_mm;
}

/* the fragment being written: its reads as fetched */
typedef struct {
	const char *name[2], *text[2], *qual[2];
	int len[2];
} frag_in;

/* one thread's output text of the current fragment */
typedef struct {
	char *buf;
	size_t len, cap;
} tbuf;

static int tb_reserve(tbuf *b, size_t n)
{
	if (b->len + n <= b->cap) return 0;
	size_t nc = b->cap ? b->cap : 8192;
	while (b->len + n > nc) nc *= 2;
	char *nb = realloc(b->buf, nc);
	if (!nb) return SVG_E_NOMEM;
	b->buf = nb;
	b->cap = nc;
	return 0;
}

typedef struct {
	svg_sam_writer *sink;
	svg_realign_emit_fn emit;
	void *emit_arg;
} out_t;

/* write_single_fragment, core.c:1888-2178 (base space): the SAM record(s) of one location */
static int write_fragment(const svg_realign *ra, tally_t *T, const out_t *O, tbuf *tb, outrec *rec1, outrec *rec2,
                          int all_locations, int loc, const frag_in *F, int64_t pair_number, int ok1, int ok2)
{
	const svg_realign_params *p = &ra->p;
	const svg_genome_arrays *g = ra->g;
	int tlen = 0;
	if (ok1 && ok2 && rec1->chr == rec2->chr) tlen = calc_tlen(rec1, rec2, F->len[0], F->len[1]);
	const int flag1 = calc_flags(ra, T, rec1, rec2, 0, loc, tlen, ok1, ok2);
	int flag2 = -1;
	if (p->paired) {
		flag2 = calc_flags(ra, T, rec1, rec2, 1, loc, tlen, ok2, ok1);
		if (loc == 0 && (flag2 & S_PROPER)) T->st.all_correct_PE_reads++;
	}
	/* the read texts and qualities, reversed when the record (or, without one, R2) says so */
	char seq[2][MAXRL + 2], qual[2][MAXRL + 2], name[2][256];
	const int ends = 1 + (p->paired != 0);
	for (int e = 0; e < ends; e++) {
		const outrec *cr = e ? rec2 : rec1;
		const int rev = cr ? cr->strand : e;   /* calc_should_reverse, core.c:1791-1803 */
		const int L = F->len[e];
		if (rev) {
			revcomp(seq[e], F->text[e], L);
			if (F->qual[e][0]) revstr(qual[e], F->qual[e], L);
			else qual[e][0] = 0;
		} else {
			memcpy(seq[e], F->text[e], (size_t)L);
			seq[e][L] = 0;
			snprintf(qual[e], sizeof qual[e], "%s", F->qual[e]);
		}
		if (p->phred_offset == 64 && qual[e][0])   /* fastq_64_to_33 (core.c:2590-2594) */
			for (char *q = qual[e]; *q; q++) *q = (char)(*q - 31);
		snprintf(name[e], sizeof name[e], "%s", F->name[e]);
		char *sl = strchr(name[e], '/');   /* remove_backslash, subread.h:251 */
		if (sl) *sl = 0;
	}
	if (!qual[0][0]) {   /* FASTA input: 'I' for every base (core.c:2011-2019) */
		for (int e = 0; e < ends; e++) {
			int k;
			for (k = 0; seq[e][k]; k++) qual[e][k] = 'I';
			qual[e][k] = 0;
		}
	}
	char tags[2][1000 + ADD_INFO_LEN];
	int tp[2] = {0, 0};
	tags[0][0] = tags[1][0] = 0;
	if (ok1 || ok2) {
		tp[0] = snprintf(tags[0], 310, "HI:i:%d\tNH:i:%d", loc + 1, all_locations);
		tp[1] = snprintf(tags[1], 310, "HI:i:%d\tNH:i:%d", loc + 1, all_locations);
	}
	if (p->read_group_id[0]) {
		tp[0] += snprintf(tags[0] + tp[0], 310, "\tRG:Z:%s", p->read_group_id);
		tp[1] += snprintf(tags[1] + tp[1], 310, "\tRG:Z:%s", p->read_group_id);
	}
	const char *chro[2] = {"*", "*"}, *cig[2] = {"*", "*"};
	int okv[2] = {ok1, ok2};
	outrec *rv[2] = {rec1, rec2};
	for (int e = 0; e < ends; e++)
		if (okv[e]) {
			/* additional_information: XS (convert_read_to_tmp), then NM (core.c:2029-2039) */
			tp[e] += snprintf(tags[e] + tp[e], sizeof tags[e] - (size_t)tp[e], "%s\tNM:i:%d", rv[e]->info,
			                  (int)(int16_t)edit_dist(rv[e]->cigar, rv[e]->res->final_mismatched));
			chro[e] = g->chr_name + (size_t)rv[e]->chr * SVG_CHR_NAME_LEN;
			cig[e] = rv[e]->cigar;
		}
	long long otl[2] = {tlen, tlen};
	if (ok1 && ok2) {
		if (rec1->offset > rec2->offset) otl[0] = -otl[0];
		else if (rec2->offset > rec1->offset) otl[1] = -otl[1];
		else if (rec1->strand) otl[0] = -otl[0];
		else otl[1] = -otl[1];
	}
	if (loc == 0) {
		if (p->paired) { if (ok1 || ok2) T->st.all_mapped_reads++; }
		else if (ok1) T->st.all_mapped_reads++;
	}
	int opos[2] = {0, 0}, omq[2] = {0, 0};
	for (int e = 0; e < 2; e++)
		if (okv[e]) {
			opos[e] = imax(1, rv[e]->offset);
			omq[e] = rv[e]->mapq;
		}
	const char *mate[2] = {chro[1], chro[0]};
	if (chro[0] == chro[1] && chro[0][0] != '*') mate[0] = mate[1] = "=";
	svg_sam_record sr[2];
	for (int e = 0; e < ends; e++) {
		sr[e].qname = name[e];
		sr[e].flag = e ? flag2 : flag1;
		sr[e].rname = chro[e];
		sr[e].pos = (uint32_t)opos[e];
		sr[e].mapq = omq[e];
		sr[e].cigar = cig[e];
		sr[e].rnext = mate[e];
		sr[e].pnext = (uint32_t)opos[1 - e];
		sr[e].tlen = (int32_t)otl[e];
		sr[e].seq = seq[e];
		sr[e].qual = qual[e];
		sr[e].tags = tags[e];
	}
	if (O->sink) {
		/* SAM lines, or (BAM sink) the records in BAM form: refID = the contig's index in the header,
		 * the mate's the other end's ('=' and '*' included: '*' is -1) */
		const int bam = svg_sam_writer_is_bam(O->sink);
		size_t need = 1024;
		for (int e = 0; e < ends; e++)
			need += strlen(name[e]) + strlen(chro[e]) + strlen(cig[e]) + 2 * (size_t)F->len[e] + strlen(tags[e]) + 80 + (bam ? 4 * 96 : 0);
		if (tb_reserve(tb, need)) { svg_set_error("out of memory"); return SVG_E_NOMEM; }
		for (int e = 0; e < ends; e++) {
			const int32_t ref = okv[e] ? (int32_t)rv[e]->chr : -1, mref = okv[1 - e] ? (int32_t)rv[1 - e]->chr : -1;
			const int64_t n = bam ? svg_bam_format(&sr[e], ref, mref, F->len[e], tb->buf + tb->len, tb->cap - tb->len)
			                      : svg_sam_format(&sr[e], tb->buf + tb->len, tb->cap - tb->len);
			if (n < 0) {
				svg_set_error("svg_realign_chunk: the %s record of fragment %lld does not fit", bam ? "BAM" : "SAM", (long long)pair_number);
				return SVG_E_ARG;
			}
			tb->len += (size_t)n;
		}
		return 0;
	}
	O->emit(O->emit_arg, pair_number, all_locations, loc, &sr[0], ends == 2 ? &sr[1] : NULL);
	return 0;
}

/* add_realignment_event_support, core.c:2364-2379 */
static void add_support(tally_t *T, const realign_t *res)
{
	for (int k = 0; k < MAX_EV_READ; k++) {
		const int32_t id = res->support[k];
		if (id < 0) break;
		T->ev_count[id]++;
		if (res->flank_l[k] > T->ev_fl[id]) T->ev_fl[id] = res->flank_l[k];
		if (res->flank_r[k] > T->ev_fr[id]) T->ev_fr[id] = res->flank_r[k];
	}
}

/* write_realignments_for_fragment, core.c:2383-2437 */
static int write_realignments(const svg_realign *ra, tally_t *T, const out_t *O, tbuf *tb, svg_mapping_result *records,
                              const realign_t *res1, const realign_t *res2, const frag_in *F, int64_t pair_number, int multi_n,
                              int multi_i, int *written)
{
	const svg_realign_params *p = &ra->p;
	int ok1 = 0, ok2 = 0;
	outrec r1, r2;
	memset(&r1, 0, sizeof r1);
	memset(&r2, 0, sizeof r2);
	r1.chr = r2.chr = -1;
	if (res1) {
		ok1 = convert_rec(ra, res1, &records[res1->rec], F->len[0], &r1);
		if (ok1) add_support(T, res1);
	}
	if (res2) {
		ok2 = convert_rec(ra, res2, &records[res2->rec], F->len[1], &r2);
		if (ok2) add_support(T, res2);
	}
	if (multi_i < 1) {
		if (!ok1 && !ok2) T->st.all_unmapped_reads++;
		else if (!ok1 || !ok2) {
			T->st.not_properly_pairs_only_one_end_mapped++;
			if ((ok1 && (res1->realign_flags & F_BREAKEVEN)) || (ok2 && (res2->realign_flags & F_BREAKEVEN))) T->st.all_multimapping_reads++;
			else T->st.all_uniquely_mapped_reads++;
		} else {
			if (res1->realign_flags & F_BREAKEVEN) T->st.all_multimapping_reads++;
			else T->st.all_uniquely_mapped_reads++;
		}
	}
	int rc = 0;
	if (!p->ignore_unmapped_reads || ok1 || ok2) {
		rc = write_fragment(ra, T, O, tb, res1 ? &r1 : NULL, res2 ? &r2 : NULL, multi_n, multi_i, F, pair_number, ok1, ok2);
		(*written)++;
		/* core.c:2175-2176 */
		if (ok1) records[res1->rec].selected_position += (uint32_t)r1.soft;
		if (ok2) records[res2->rec].selected_position += (uint32_t)r2.soft;
	}
	return rc;
}

/* locate_current_value_index, core.c:2216-2249: NULL = the record is outside every block */
static const garray *record_block(const svg_genome_arrays *g, const svg_mapping_result *r, int rlen)
{
	if (g->nblocks < 2) {
		const uint32_t b = g->blk[0].start_base_offset, e = g->blk[0].start_base_offset + g->blk[0].length;
		if (r->selected_position >= b && r->selected_position + (uint32_t)rlen <= e) return &g->blk[0];
		return NULL;
	}
	for (int k = 0; k < g->nblocks; k++) {
		const uint32_t b = g->blk[k].start_base_offset, e = g->blk[k].start_base_offset + g->blk[k].length;
		const uint32_t sp = r->selected_position;
		if ((k == 0 && sp >= b && sp < e - 1000000u) || (k > 0 && k < g->nblocks - 1 && sp >= b + 1000000u && sp < e - 1000000u) ||
		    (k == g->nblocks - 1 && sp >= b + 1000000u && sp < e))
			return &g->blk[k];
	}
	return NULL;
}

/* calc_end_pos (core.c:4755-4779, no exonic bitmap) and test_PE_and_same_chro_cigars
 * (core.c:4781-4811) */
static uint32_t calc_end_pos(uint32_t p0, const char *cigar, uint32_t *skipped)
{
	uint32_t cursor = p0, tmpi = 0;
	for (int c = 0; cigar[c]; c++) {
		const int nch = cigar[c];
		if (is_digit(nch)) tmpi = tmpi * 10 + (uint32_t)(nch - '0');
		else {
			if ((nch == 'S' && cursor == p0) || nch == 'M' || nch == 'N' || nch == 'D') {
				cursor += tmpi;
				if (nch == 'N' || nch == 'D') *skipped += tmpi;
			}
			tmpi = 0;
		}
	}
	return cursor;
}

static void test_pe(const svg_realign *ra, const realign_t *a, const realign_t *b, int *is_exonic, int *is_pe, int *same_chro, int *res_tlen)
{
	int c1, c2, p1, p2;
	*same_chro = 0;
	*is_pe = 0;
	*is_exonic = 1;
	locate_max(ra->g, a->first_base_position, &c1, &p1, NULL, NULL, 0);
	locate_max(ra->g, b->first_base_position, &c2, &p2, NULL, NULL, 0);
	if (c1 == c2) {
		uint32_t s1 = 0, s2 = 0;
		const uint32_t e1 = calc_end_pos(a->first_base_position, a->cigar, &s1);
		const uint32_t e2 = calc_end_pos(b->first_base_position, b->cigar, &s2);
		uint32_t tlen = (e1 > e2 ? e1 : e2) - (a->first_base_position < b->first_base_position ? a->first_base_position : b->first_base_position);
		if (tlen > s1) tlen -= s1;
		if (tlen > s2) tlen -= s2;
		*same_chro = 1;
		if (tlen >= (uint32_t)ra->p.min_pair_distance && tlen <= (uint32_t)ra->p.max_pair_distance) *is_pe = 1;
		*res_tlen = (int)tlen;
	} else {
		*res_tlen = 0x7fffffff;
		*is_exonic = 0;
	}
}

/* add_repeated_buffer, core.c:2443-2485 */
typedef struct { uint32_t pos[2]; const char *cig[2]; } rep_ent;
static int add_repeated(rep_ent *buf, int *count, int cap, const realign_t *r1, const realign_t *r2)
{
	const char *c1 = r1 ? r1->cigar : "*", *c2 = r2 ? r2->cigar : "*";
	const uint32_t p1 = r1 ? r1->first_base_position : 0, p2 = r2 ? r2->first_base_position : 0;
	for (int k = 0; k < *count; k++)
		if (buf[k].pos[0] == p1 && buf[k].pos[1] == p2 && !strcmp(buf[k].cig[0], c1) && !strcmp(buf[k].cig[1], c2)) return 1;
	if (*count < cap) {
		buf[*count].pos[0] = p1;
		buf[*count].pos[1] = p2;
		buf[*count].cig[0] = c1;
		buf[*count].cig[1] = c2;
		(*count)++;
	}
	return 0;
}

/* one worker's scratch */
typedef struct {
	wk_t W;
	rtext rt[2][2];                 /* [end][negative strand] */
	realign_t *finals;              /* [(end + 2 * best) * MAX_ALN + i] */
	int *cand_idx[2], *cand_match[2], *cand_mm[2], *cand_pen[2];
	unsigned long long *score;
	int *tlen_buf;
	rep_ent *rep;
	tally_t T;
	tbuf tb;
} worker_t;

/* do_iteration_two's per-fragment body, core.c:2551-2975.  tlen_seq: the expected-TLEN state may
 * change (the caller runs such fragments in order, on one thread) */
static int do_fragment(svg_realign *ra, worker_t *wk, const svg_fragment_reads *R, svg_mapping_result *records, int64_t r,
                       const out_t *O)
{
	const svg_realign_params *p = &ra->p;
	const int ends = 1 + (p->paired != 0), mb = p->multi_best;
	const int cap_cand = mb * MAX_ALN;
	wk_t *W = &wk->W;
	frag_in F;
	for (int e = 0; e < ends; e++) {
		const uint64_t k = (uint64_t)r * (uint64_t)ends + (uint64_t)e;
		F.name[e] = R->buf + R->name_off[k];
		F.text[e] = R->buf + R->text_off[k];
		F.qual[e] = R->buf + R->qual_off[k];
		F.len[e] = R->len[k];
		if (F.len[e] > MAXRL) F.len[e] = MAXRL;
	}
	if (ends == 1) { F.name[1] = F.text[1] = F.qual[1] = ""; F.len[1] = 0; }
	svg_mapping_result *rec = records + (uint64_t)r * (uint64_t)(ends * mb);
	int max_votes = rec[0].selected_votes;
	if (ends == 2) max_votes = imax(rec[0].selected_votes, rec[mb].selected_votes);
	int ncand[2] = {0, 0}, step2[2] = {0, 0};
	int built[2][2] = {{0, 0}, {0, 0}};
	int rep_count = 0;
	const int rep_cap = MAX_ALN * p->reported_multi_best;   /* entries of two slots each (core.c:2472) */
	for (int e = 0; e < ends; e++) {
		for (int b = 0; b < mb; b++) {
			svg_mapping_result *cur = &rec[e * mb + b];
			if (cur->selected_votes < p->min_votes_second || max_votes < p->min_votes_first) {
				cur->selected_votes = 0;
				continue;
			}
			const garray *vi = record_block(ra->g, cur, F.len[e]);
			if (!vi) { cur->selected_votes = 0; continue; }
			const int neg = (cur->result_flags & F_NEG) ? 1 : 0;
			if (!built[e][neg]) {
				if (neg) {
					char tmp[MAXRL + 2];
					revcomp(tmp, F.text[e], F.len[e]);
					rtext_build(&wk->rt[e][1], tmp, F.len[e]);
				} else rtext_build(&wk->rt[e][0], F.text[e], F.len[e]);
				built[e][neg] = 1;
			}
			cur->result_flags &= (int16_t)~F_FULLY;
			step2[e] = b + 1;
			W->vi = vi;
			W->t = &wk->rt[e][neg];
			realign_t *fin = wk->finals + (size_t)(e + 2 * b) * MAX_ALN;
			const int nf = explain_read(W, cur, (int)((uint64_t)r * (uint64_t)(ends * mb) + (uint64_t)(e * mb + b)), F.len[e], fin);
			for (int i = 0; i < nf; i++) {
				if (ncand[e] >= cap_cand) break;
				if ((cur->result_flags & F_FULLY) && fin[i].final_matched > 0) {
					const int c = ncand[e]++;
					wk->cand_pen[e][c] = fin[i].final_penalty;
					wk->cand_match[e][c] = fin[i].final_matched;
					wk->cand_mm[e][c] = fin[i].final_mismatched;
					wk->cand_idx[e][c] = (e + 2 * b) * MAX_ALN + i;
				}
			}
		}
	}
	const int need_expect_tlen = ncand[1] && ncand[0] && p->reported_multi_best < 2 && ra->tlen_n < TLEN_PAIRS;
	int out_cursor = 0, written = 0, rc = 0;
	if (ncand[1] == 0 || ncand[0] == 0) {
		int occ = 0;
		for (int e = 0; e < ends; e++) {
			const int nc = ncand[e];
			if (nc <= 0) continue;
			unsigned long long best = 0, scores[64];
			for (int i = 0; i < nc; i++) {
				const realign_t *cr = &wk->finals[wk->cand_idx[e][i]];
				const unsigned int m = (unsigned)wk->cand_match[e][i], mm = (unsigned)wk->cand_mm[e][i], pen = (unsigned)wk->cand_pen[e][i];
				unsigned long long s;
				if (p->experiment_type == SVG_EXPERIMENT_DNASEQ) s = m * 100000llu + (10000 - mm);
				else s = ((100000llu * (10000 - mm) + m) * 50llu - pen) * 20llu + (unsigned long long)(long long)cr->known_junction_supp;
				if (s > best) best = s;
				scores[i] = s;
			}
			for (int i = 0; i < nc; i++) {
				const realign_t *cr = &wk->finals[wk->cand_idx[e][i]];
				if (scores[i] >= best && !(cr->realign_flags & F_TOO_MANY)) {
					if (add_repeated(wk->rep, &rep_count, rep_cap, e ? NULL : cr, e ? cr : NULL)) scores[i] = 0;
					else occ++;
				}
			}
			if (occ < 2 || p->report_multi_mapping) {
				const int breakeven = occ > 1;
				occ = imin(occ, p->reported_multi_best);
				for (int i = 0; i < nc; i++) {
					realign_t *cr = &wk->finals[wk->cand_idx[e][i]];
					if (scores[i] >= best && !(cr->realign_flags & F_TOO_MANY) && out_cursor < p->reported_multi_best) {
						if (breakeven) cr->realign_flags |= F_BREAKEVEN;
						cr->mapq_adjustment = (int16_t)(wk->cand_mm[e][i] + step2[e]);
						rc |= write_realignments(ra, &wk->T, O, &wk->tb, records, e ? NULL : cr, e ? cr : NULL, &F, r, occ, out_cursor,
						                         &written);
						out_cursor++;
					}
				}
			}
		}
	} else {
		int occ = 0;
		int expected_tlen;
		if (ra->tlen_n >= TLEN_PAIRS) expected_tlen = (int)(ra->tlen_sum / ra->tlen_n);
		else expected_tlen = (p->min_pair_distance + p->max_pair_distance) / 2;
		unsigned long long highest = 0;
		const int stride = mb * MAX_ALN;
		if (need_expect_tlen) memset(wk->tlen_buf, 0, sizeof(int) * (size_t)stride * (size_t)stride);
		memset(wk->score, 0, sizeof(unsigned long long) * (size_t)stride * (size_t)stride);
		for (int i1 = 0; i1 < ncand[0]; i1++) {
			if (wk->cand_match[0][i1] < 1) continue;
			const realign_t *a = &wk->finals[wk->cand_idx[0][i1]];
			for (int i2 = 0; i2 < ncand[1]; i2++) {
				if (wk->cand_match[1][i2] < 1) continue;
				const realign_t *b = &wk->finals[wk->cand_idx[1][i2]];
				int is_pe = 0, tlen = 0, same_chro = 0, is_exonic = 0;
				unsigned long long fs = 0;
				test_pe(ra, a, b, &is_exonic, &is_pe, &same_chro, &tlen);
				unsigned long long tlen_score = 0;
				if (is_pe && p->no_tlen_preference == 0 && p->reported_multi_best < 2) {
					tlen_score = (unsigned long long)(long long)(tlen > expected_tlen ? tlen - expected_tlen : expected_tlen - tlen);
					tlen_score = tlen_score > 999 ? 0 : 999 - tlen_score;
				}
				if (p->experiment_type == SVG_EXPERIMENT_DNASEQ) {
					const int weight = is_pe ? 120 : same_chro ? 100 : 80;
					fs = (unsigned long long)(long long)(weight * (wk->cand_match[0][i1] + wk->cand_match[1][i2]));
					fs = fs * 1000llu - (unsigned long long)(long long)wk->cand_mm[0][i1] - (unsigned long long)(long long)wk->cand_mm[1][i2];
					fs = fs * 20llu - (unsigned long long)(long long)wk->cand_pen[0][i1] - (unsigned long long)(long long)wk->cand_pen[1][i2];
					fs = fs * 1000llu + tlen_score;
				} else {
					int weight;
					if (is_exonic && is_pe) weight = 5000;
					else if (is_pe || is_exonic) weight = 3000;
					else if (same_chro) weight = 1000;
					else weight = 300;
					fs = (unsigned long long)(long long)(weight / (wk->cand_mm[0][i1] + wk->cand_mm[1][i2] + 1 + 2));
					fs = fs * 3000llu + (unsigned long long)(long long)(wk->cand_match[0][i1] + wk->cand_match[1][i2]);
					fs = fs * 20 + (unsigned long long)(long long)b->known_junction_supp + (unsigned long long)(long long)a->known_junction_supp;
					fs = fs * 20 - (unsigned long long)(long long)wk->cand_pen[0][i1] - (unsigned long long)(long long)wk->cand_pen[1][i2];
					fs = fs * 1000 + tlen_score;
				}
				if (is_pe && need_expect_tlen) wk->tlen_buf[i1 * stride + i2] = tlen;
				wk->score[i1 * stride + i2] = fs;
				if (fs > highest) {
					occ = 1;
					highest = fs;
					rep_count = 0;
					add_repeated(wk->rep, &rep_count, rep_cap, a, b);
				} else if (fs == highest) {
					int is_rep = 0;
					if (p->reported_multi_best) is_rep = add_repeated(wk->rep, &rep_count, rep_cap, a, b);
					if (is_rep) wk->score[i1 * stride + i2] = 0;
					else occ++;
				}
			}
		}
		if (occ <= 1 || p->report_multi_mapping) {
			const int breakeven = occ > 1;
			occ = imin(occ, p->reported_multi_best);
			for (int i1 = 0; i1 < ncand[0]; i1++) {
				if (wk->cand_match[0][i1] < 1) continue;
				for (int i2 = 0; i2 < ncand[1]; i2++) {
					if (wk->cand_match[1][i2] < 1) continue;
					if (wk->score[i1 * stride + i2] == highest && out_cursor < p->reported_multi_best) {
						if (need_expect_tlen) {
							const int this_tlen = wk->tlen_buf[i1 * stride + i2];
							if (this_tlen > 0) {
								ra->tlen_n++;
								ra->tlen_sum += this_tlen;
							}
						}
						realign_t *a = &wk->finals[wk->cand_idx[0][i1]], *b = &wk->finals[wk->cand_idx[1][i2]];
						if (breakeven) { a->realign_flags |= F_BREAKEVEN; b->realign_flags |= F_BREAKEVEN; }
						a->mapq_adjustment = (int16_t)(step2[0] + wk->cand_mm[0][i1]);
						b->mapq_adjustment = (int16_t)(step2[1] + wk->cand_mm[1][i2]);
						rc |= write_realignments(ra, &wk->T, O, &wk->tb, records, a, b, &F, r, occ, out_cursor, &written);
						out_cursor++;
					}
				}
			}
		}
	}
	if (out_cursor < 1) rc |= write_realignments(ra, &wk->T, O, &wk->tb, records, NULL, NULL, &F, r, 0, 0, &written);
	if (rc) return rc < 0 ? rc : SVG_E_ARG;
	return 0;
}

/* fragments [b, e) by one worker: their text (every location, in order) goes to the sink in one
 * put (a fragment that writes nothing still moves the order on) */
static int do_fragments(svg_realign *ra, worker_t *wk, const svg_fragment_reads *R, svg_mapping_result *records, int64_t b, int64_t e,
                        const out_t *O)
{
	wk->tb.len = 0;
	for (int64_t r = b; r < e; r++) {
		const int rc = do_fragment(ra, wk, R, records, r, O);
		if (rc) return rc;
	}
	if (O->sink) return svg_sam_writer_put_block(O->sink, b, e - b, wk->tb.buf ? wk->tb.buf : "", wk->tb.len);
	return 0;
}

int svg_realign_create(const svg_genome_arrays *g, const svg_realign_params *p, svg_realign **out)
{
	if (!g || !p || !out) { svg_set_error("svg_realign_create: NULL argument"); return SVG_E_ARG; }
	*out = NULL;
	if (p->do_fusion_detection || p->do_long_del_detection || p->color_space || p->exonic_region_bitmap || p->scrna_input_mode ||
	    p->do_big_margin_filtering_for_reads) {
		svg_set_error("svg_realign_create: configuration not supported (fusion / long-deletion detection, colour space, "
		              "exonic-region scoring, scRNA mode or big-margin read filtering)");
		return SVG_E_UNSUPPORTED;
	}
	if (p->multi_best < 1 || p->multi_best > 16 || p->reported_multi_best < 0 || p->reported_multi_best > 16) {
		svg_set_error("svg_realign_create: multi_best %d / reported %d out of range", p->multi_best, p->reported_multi_best);
		return SVG_E_ARG;
	}
	svg_realign *ra = calloc(1, sizeof *ra);
	if (!ra) { svg_set_error("out of memory"); return SVG_E_NOMEM; }
	ra->p = *p;
	ra->g = g;
	ra->bm_small = calloc(BM_WORDS, sizeof(uint64_t));
	ra->bm_large = calloc(BM_WORDS, sizeof(uint64_t));
	if (!ra->bm_small || !ra->bm_large) { svg_realign_destroy(ra); svg_set_error("out of memory"); return SVG_E_NOMEM; }
	pthread_once(&revc_once, revc_init);
	*out = ra;
	return 0;
}

void svg_realign_destroy(svg_realign *ra)
{
	if (!ra) return;
	free(ra->ev); free(ra->site); free(ra->ids); free(ra->bm_small); free(ra->bm_large);
	free(ra);
}

static void worker_free(worker_t *w)
{
	if (!w) return;
	free(w->finals);
	for (int e = 0; e < 2; e++) { free(w->cand_idx[e]); free(w->cand_match[e]); free(w->cand_mm[e]); free(w->cand_pen[e]); }
	free(w->score); free(w->tlen_buf); free(w->rep);
	free(w->T.ev_count); free(w->T.ev_fl); free(w->T.ev_fr);
	free(w->tb.buf);
	free(w);
}

static worker_t *worker_new(const svg_realign *ra)
{
	const int mb = ra->p.multi_best, nc = mb * MAX_ALN;
	worker_t *w = calloc(1, sizeof *w);
	if (!w) return NULL;
	w->W.ra = ra;
	w->finals = calloc((size_t)(2 * mb * MAX_ALN), sizeof(realign_t));
	for (int e = 0; e < 2; e++) {
		w->cand_idx[e] = calloc((size_t)nc, sizeof(int));
		w->cand_match[e] = calloc((size_t)nc, sizeof(int));
		w->cand_mm[e] = calloc((size_t)nc, sizeof(int));
		w->cand_pen[e] = calloc((size_t)nc, sizeof(int));
	}
	w->score = calloc((size_t)nc * (size_t)nc, sizeof(unsigned long long));
	w->tlen_buf = calloc((size_t)nc * (size_t)nc, sizeof(int));
	w->rep = calloc((size_t)(MAX_ALN * 2 * (ra->p.reported_multi_best + 1)), sizeof(rep_ent));
	const size_t ne = (size_t)(ra->n_ev > 0 ? ra->n_ev : 1);
	w->T.ev_count = calloc(ne, sizeof(uint32_t));
	w->T.ev_fl = malloc(ne * sizeof(int16_t));
	w->T.ev_fr = malloc(ne * sizeof(int16_t));
	if (!w->finals || !w->score || !w->tlen_buf || !w->rep || !w->T.ev_count || !w->T.ev_fl || !w->T.ev_fr || !w->cand_idx[1] ||
	    !w->cand_pen[1]) {
		worker_free(w);
		return NULL;
	}
	for (size_t i = 0; i < ne; i++) w->T.ev_fl[i] = w->T.ev_fr[i] = INT16_MIN;
	return w;
}

typedef struct {
	svg_realign *ra;
	const svg_fragment_reads *R;
	svg_mapping_result *records;
	const out_t *O;
	worker_t *wk;
	int64_t *next, end;
	volatile int *rc;
	char *err;              /* the first failing worker's svg_last_error() (errors are per thread) */
} job_t;

#define BLOCK 256

static void *worker_run(void *v)
{
	job_t *j = v;
	for (;;) {
		if (*j->rc) break;
		const int64_t b = __atomic_fetch_add(j->next, BLOCK, __ATOMIC_RELAXED);
		if (b >= j->end) break;
		const int64_t e = b + BLOCK < j->end ? b + BLOCK : j->end;
		const int rc = do_fragments(j->ra, j->wk, j->R, j->records, b, e, j->O);
		if (rc) {
			int zero = 0;
			if (__atomic_compare_exchange_n(j->rc, &zero, rc, 0, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED))
				snprintf(j->err, 256, "%s", svg_last_error());
			break;
		}
	}
	return NULL;
}

int svg_realign_chunk(svg_realign *ra, const svg_fragment_reads *R, svg_mapping_result *records, svg_sam_writer *sink,
                      svg_realign_emit_fn emit, void *emit_arg, int threads, svg_realign_stats *stats)
{
	if (!ra || !R || (R->n && (!records || !R->buf || !R->name_off || !R->text_off || !R->qual_off || !R->len)) || (!sink && !emit)) {
		svg_set_error("svg_realign_chunk: bad argument");
		return SVG_E_ARG;
	}
	if (threads <= 0) threads = svg_host_threads();
	if (!sink) threads = 1;   /* the callback sees the fragments in order from one thread */
	if (threads > 64) threads = 64;
	const out_t O = {sink, emit, emit_arg};
	worker_t *wk[64] = {0};
	const double t0 = now_s();
	int rc = 0;
	for (int t = 0; t < threads; t++)
		if (!(wk[t] = worker_new(ra))) { rc = SVG_E_NOMEM; svg_set_error("out of memory"); break; }
	int64_t r = 0;
	/* fragments that can move the expected-TLEN estimate go in order on one thread (do_iteration_two
	 * reads and updates global_context->expected_TLEN_* as it goes, core.c:2705,2792-2794,2927-2936) */
	const int tlen_seq = ra->p.paired && ra->p.reported_multi_best < 2;
	while (!rc && r < (int64_t)R->n && tlen_seq && ra->tlen_n < TLEN_PAIRS) {
		rc = do_fragments(ra, wk[0], R, records, r, r + 1, &O);
		r++;
	}
	const double t1 = now_s();
	if (!rc && r < (int64_t)R->n) {
		int64_t next = r;
		volatile int jrc = 0;
		char jerr[256] = "";
		job_t jobs[64];
		pthread_t th[64];
		int started = 0;
		for (int t = 0; t < threads; t++) {
			jobs[t] = (job_t){ra, R, records, &O, wk[t], &next, (int64_t)R->n, &jrc, jerr};
			if (t == 0) continue;
			if (pthread_create(&th[t], NULL, worker_run, &jobs[t])) break;
			started = t;
		}
		worker_run(&jobs[0]);
		for (int t = 1; t <= started; t++) pthread_join(th[t], NULL);
		rc = jrc;
		if (rc) svg_set_error("%s", jerr);
	}
	const double t2 = now_s();
	/* the counters and the event support of every worker */
	for (int t = 0; t < threads && wk[t]; t++) {
		const worker_t *w = wk[t];
		if (stats) {
			stats->all_mapped_reads += w->T.st.all_mapped_reads;
			stats->all_correct_PE_reads += w->T.st.all_correct_PE_reads;
			stats->not_properly_pairs_wrong_arrangement += w->T.st.not_properly_pairs_wrong_arrangement;
			stats->not_properly_pairs_different_chro += w->T.st.not_properly_pairs_different_chro;
			stats->not_properly_different_strands += w->T.st.not_properly_different_strands;
			stats->not_properly_pairs_TLEN_wrong += w->T.st.not_properly_pairs_TLEN_wrong;
			stats->all_unmapped_reads += w->T.st.all_unmapped_reads;
			stats->not_properly_pairs_only_one_end_mapped += w->T.st.not_properly_pairs_only_one_end_mapped;
			stats->all_multimapping_reads += w->T.st.all_multimapping_reads;
			stats->all_uniquely_mapped_reads += w->T.st.all_uniquely_mapped_reads;
		}
		for (int64_t i = 0; i < ra->n_ev; i++) {
			svg_event *e = &ra->ev[i];
			if (w->T.ev_count[i]) e->final_counted_reads = (uint16_t)(e->final_counted_reads + w->T.ev_count[i]);
			if (w->T.ev_fl[i] > e->junction_flanking_left) e->junction_flanking_left = w->T.ev_fl[i];
			if (w->T.ev_fr[i] > e->junction_flanking_right) e->junction_flanking_right = w->T.ev_fr[i];
		}
	}
	for (int t = 0; t < threads; t++) worker_free(wk[t]);
	if (svg_get_option("debug") & 16)
		fprintf(stderr, "svg_realign_chunk: %llu fragments, %d threads: setup+ordered %.4f s (%lld in order), parallel %.4f s, merge %.4f s\n",
		        (unsigned long long)R->n, threads, t1 - t0, (long long)r, t2 - t1, now_s() - t2);
	return rc;
}
