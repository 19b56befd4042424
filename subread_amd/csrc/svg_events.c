/*
 * svg_events.c -- host post-vote stage: indel and junction events from the vote records
 * (the final-run tail of do_voting, core.c:3241-3290) and the table merge of
 * finalise_indel_and_junction_thread (core-indel.c:1012-1141).  See include/subread_events.h.
 *
 * Event table: a growable array of events plus an open-addressing map from a coordinate to
 * the ids of the events that have it as small or large side -- an id list of put_new_event's
 * shape (core-indel.c:1385-1419): room for 9 entries (EVENT_ENTRIES_INIT_SIZE), of which a put
 * fills at most 8 (it keeps a 0 after the last); a list given by svg_events_load_sites may have
 * less room (sort_junction_entry_table sizes its lists to their entries, core-indel.c:897-906).
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <pthread.h>
#include <string.h>
#include <stdint.h>
#include "subread_vote.h"
#include "subread_events.h"
#include "svg_internal.h"

#define EV_PER_SITE        9          /* entries of an id list (EVENT_ENTRIES_INIT_SIZE, MAX_EVENT_ENTRIES_PER_SITE) */
#define MAX_INDEL_SECT     7          /* MAX_INDEL_SECTIONS: the loop bound of find_new_indels */
#define LONG_READ          160        /* EXON_LONG_READ_LENGTH */
#define MAX_INSERTION      200        /* MAX_INSERTION_LENGTH */
#define GAPPED_FLAG        64         /* CORE_IS_GAPPED_READ */
#define JUMPED_FLAG        4          /* CORE_IS_STRAND_JUMPED */
#define NEG_FLAG           SVG_NEGATIVE_STRAND_FLAG
#define MASK_MATCH         0          /* INDEL_MASK_BY_*, core-indel.c:4560-4563 */
#define MASK_INSERTION     1
#define MASK_DELETION      2
#define MASK_MISMATCH      3

void svg_event_params_default(svg_event_params *e)
{
	e->dp_penalty_create_gap = -1;
	e->dp_penalty_extend_gap = 0;
	e->dp_match_score = 2;
	e->dp_mismatch_penalty = 0;
	e->report_multi_mapping_reads = 0;
	e->quality_base = '#';
	e->maximise_sensitivity_indel = 0;
}

/* ------------------------------------------------------------------ base arrays */
/* (garray and struct svg_genome_arrays are in svg_internal.h: svg_realign.c reads them too) */
void svg_genome_arrays_close(svg_genome_arrays *g)
{
	int b;
	if (!g) return;
	if (g->owned)
		for (b = 0; b < g->nblocks; b++) free(g->blk[b].values);
	free(g->blk);
	free(g->chr_end);
	free(g->chr_name);
	free(g);
}

int svg_genome_arrays_wrap(const svg_value_block *blocks, int nblocks, const uint32_t *chr_end, const char *names,
                           int name_stride, uint32_t n_chr, int padding, int gap, svg_genome_arrays **out)
{
	if (!blocks || nblocks < 1 || !chr_end || !out || (n_chr && !names) || name_stride < 1) {
		svg_set_error("svg_genome_arrays_wrap: bad argument");
		return SVG_E_ARG;
	}
	svg_genome_arrays *g = calloc(1, sizeof *g);
	if (!g) { svg_set_error("out of memory"); return SVG_E_NOMEM; }
	g->blk = calloc((size_t)nblocks, sizeof(garray));
	g->chr_end = malloc(4 * ((size_t)n_chr + 1));
	g->chr_name = calloc((size_t)n_chr + 1, SVG_CHR_NAME_LEN);
	if (!g->blk || !g->chr_end || !g->chr_name) { svg_genome_arrays_close(g); svg_set_error("out of memory"); return SVG_E_NOMEM; }
	for (int b = 0; b < nblocks; b++) {
		g->blk[b].values = (uint8_t *)blocks[b].values;
		g->blk[b].start_point = blocks[b].start_point;
		g->blk[b].length = blocks[b].length;
		g->blk[b].start_base_offset = blocks[b].start_base_offset;
		g->blk[b].values_bytes = blocks[b].values_bytes;
	}
	g->nblocks = nblocks;
	g->owned = 0;
	for (uint32_t c = 0; c < n_chr; c++) {
		g->chr_end[c] = chr_end[c];
		snprintf(g->chr_name + (size_t)c * SVG_CHR_NAME_LEN, SVG_CHR_NAME_LEN, "%s", names + (size_t)c * name_stride);
	}
	g->n_chr = n_chr;
	g->padding = padding;
	g->gap = gap;
	*out = g;
	return 0;
}

int svg_genome_arrays_contigs(const svg_genome_arrays *g, uint32_t *n, const char **names, uint32_t *lengths)
{
	if (!g || !n) { svg_set_error("svg_genome_arrays_contigs: NULL argument"); return SVG_E_ARG; }
	*n = g->n_chr;
	for (uint32_t c = 0; c < g->n_chr; c++) {
		if (names) names[c] = g->chr_name + (size_t)c * SVG_CHR_NAME_LEN;
		/* FETCH_SEQ_LEN, core.c:3841 (write_sam_headers' @SQ LN): read_offsets delta + 16 - 2 * padding */
		if (lengths) lengths[c] = g->chr_end[c] - (c ? g->chr_end[c - 1] : 0) + 16u - 2u * (uint32_t)g->padding;
	}
	return 0;
}

/* gvindex_load (gene-value-index.c:190-228) per block; load_offsets' .reads table
 * (gene-algorithms.c:1293-1370) with the .tab's padding option */
int svg_genome_arrays_open(const char *prefix, svg_genome_arrays **out)
{
	char fn[4096];
	svg_genome_arrays *g;
	int b, nb;
	FILE *fp;
	if (!prefix || !out) { svg_set_error("svg_genome_arrays_open: NULL argument"); return SVG_E_ARG; }
	*out = NULL;
	nb = svg_index_count_blocks(prefix);
	if (nb < 1) { svg_set_error("index table '%s.00.b.tab' not found", prefix); return SVG_E_IO; }
	g = calloc(1, sizeof *g);
	g->blk = calloc((size_t)nb, sizeof(garray));
	g->owned = 1;
	g->padding = 1210;
	for (b = 0; b < nb; b++) {
		garray *a = &g->blk[b];
		uint32_t useful;
		snprintf(fn, sizeof fn, "%s.%02d.b.array", prefix, b);
		if (!(fp = fopen(fn, "rb"))) { svg_genome_arrays_close(g); svg_set_error("cannot open '%s'", fn); return SVG_E_IO; }
		if (fread(&a->start_point, 4, 1, fp) != 1 || fread(&a->length, 4, 1, fp) != 1) {
			fclose(fp); svg_genome_arrays_close(g); svg_set_error("'%s' truncated", fn); return SVG_E_FORMAT;
		}
		a->start_base_offset = a->start_point - a->start_point % 4;
		useful = (a->length + a->start_point - a->start_base_offset) >> 2;
		a->values_bytes = useful + 1;
		a->values = calloc((size_t)a->values_bytes + 8, 1);
		if (fread(a->values, 1, (size_t)useful + 1, fp) < useful) {
			fclose(fp); svg_genome_arrays_close(g); svg_set_error("'%s' truncated", fn); return SVG_E_FORMAT;
		}
		fclose(fp);
		g->nblocks = b + 1;
	}
	/* the padding and gap options of the first table (gehash_load_option, 0x0102 / 0x0101) */
	g->gap = 1;
	snprintf(fn, sizeof fn, "%s.00.b.tab", prefix);
	if ((fp = fopen(fn, "rb"))) {
		char magic[8];
		if (fread(magic, 1, 8, fp) == 8 && !memcmp(magic, "2subindx", 8))
			for (;;) {
				int16_t k, l, v;
				if (fread(&k, 2, 1, fp) != 1 || !k || fread(&l, 2, 1, fp) != 1) break;
				if (k == 0x0102 || k == 0x0101) {
					if (fread(&v, 2, 1, fp) != 1) break;
					if (k == 0x0102) g->padding = v; else g->gap = v;
					if (l > 2 && fseek(fp, l - 2, SEEK_CUR)) break;
					continue;
				}
				if (fseek(fp, l, SEEK_CUR)) break;
			}
		fclose(fp);
	}
	snprintf(fn, sizeof fn, "%s.reads", prefix);
	if (!(fp = fopen(fn, "r"))) { svg_genome_arrays_close(g); svg_set_error("cannot open '%s'", fn); return SVG_E_IO; }
	{
		/* load_offsets (gene-algorithms.c:1326-1368): "<end offset>\t<name>" per line, the name
		 * cut at MAX_CHROMOSOME_NAME_LEN - 1 bytes */
		char line[4096];
		uint32_t cap = 64;
		g->chr_end = malloc(4 * cap);
		g->chr_name = calloc(cap, SVG_CHR_NAME_LEN);
		while (fgets(line, sizeof line, fp)) {
			size_t ll = strlen(line);
			while (ll && (line[ll - 1] == '\n' || line[ll - 1] == '\r')) line[--ll] = 0;
			if (ll < 2) continue;
			if (g->n_chr == cap) {
				cap *= 2;
				g->chr_end = realloc(g->chr_end, 4 * cap);
				g->chr_name = realloc(g->chr_name, (size_t)cap * SVG_CHR_NAME_LEN);
			}
			g->chr_end[g->n_chr] = (uint32_t)strtoull(line, NULL, 10);
			char *tab = strchr(line, '\t');
			snprintf(g->chr_name + (size_t)g->n_chr * SVG_CHR_NAME_LEN, SVG_CHR_NAME_LEN, "%s", tab ? tab + 1 : "");
			g->n_chr++;
		}
	}
	fclose(fp);
	*out = g;
	return 0;
}

/* gvindex_get, gene-value-index.c:96-107 */
static inline char gv_get(const garray *a, uint32_t pos)
{
	uint32_t byte = (pos - a->start_base_offset) >> 2;
	if (byte >= a->values_bytes - 1) return 'N';
	return "AGCT"[(a->values[byte] >> (pos % 4 * 2)) & 3];
}

/* gvindex_get_string(buf, a, pos, 2, neg), gene-value-index.c:1118-1136 */
static void chro_2base(const garray *a, uint32_t pos, int neg, char h[2])
{
	int i;
	if (!neg) { h[0] = gv_get(a, pos); h[1] = gv_get(a, pos + 1); return; }
	for (i = 1; i >= 0; i--) {
		char c = gv_get(a, pos + 1 - (uint32_t)i);
		h[i] = c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'G' ? 'C' : c == 'C' ? 'G' : c;
	}
}

/* match_chro, gene-value-index.c:856-959 (base space, positive strand) */
static int match_chro(const char *read, const garray *a, uint32_t pos, int len)
{
	int ret = 0, i;
	uint32_t byte, bit;
	int8_t iv;
	if ((uint32_t)(pos + (uint32_t)len) >= a->length + a->start_point) return 0;
	if (pos > 0xffff0000u) return 0;
	byte = (pos - a->start_base_offset) >> 2;
	bit = pos % 4 * 2;
	if (byte >= a->values_bytes) return 0;
	iv = (int8_t)a->values[byte];
	for (i = 0; i < len; i++) {
		const int tt = (iv >> bit) & 3;
		switch (read[i]) {
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

/* match_chro_maxerror(read, a, pos, len, 0, base space, max_error 0), gene-value-index.c:1036-1088 */
static int match_exact(const char *read, const garray *a, uint32_t pos, int len)
{
	int i;
	for (i = 0; i < len; i++)
		if (read[i] != gv_get(a, pos + (uint32_t)i)) return 0;
	return len;
}

static inline int b2i(char c) { return c < 'G' ? (c == 'A' ? 0 : 2) : (c == 'G' ? 1 : 3); }

/* match_chro_range, gene-value-index.c:982-1034: the nearest 8-base exact hit of read[j..j+7]
 * (j < 4) at a byte-aligned 16-bit word of the array, searched byte by byte from pos (backwards
 * or forwards), confirmed over read_len bases; 0xffffffff when none.  The reference reads out of
 * the array for a search that starts within 500 bytes of its head (an unsigned underflow in the
 * clamp); here the search stops at the array's head instead. */
static uint32_t match_chro_range(const char *read, const garray *a, uint32_t pos, int read_len, uint32_t search_length, int back)
{
	int16_t key[4];
	int i, j;
	uint32_t offset_byte = (pos - a->start_base_offset) >> 2, dist = search_length / 4;
	for (i = 0; i < 4; i++) {
		int k = 0;
		for (j = i + 7; j >= i; j--) k = (k << 2) | b2i(read[j]);
		key[i] = (int16_t)k;
	}
	if (back) { if (dist > offset_byte - 500u) dist = offset_byte - 500u; }
	else if (dist + offset_byte >= a->values_bytes - 500u) dist = a->values_bytes - offset_byte - 501u;
	for (i = 2; (uint32_t)i < dist; i++) {
		uint64_t t = back ? (uint64_t)offset_byte - (uint64_t)i : (uint64_t)offset_byte + (uint64_t)i;
		int16_t tv;
		if (t + 1 >= (uint64_t)a->values_bytes + 8) break;   /* (see above) */
		tv = (int16_t)(a->values[t] | (a->values[t + 1] << 8));
		for (j = 0; j < 4; j++)
			if (tv == key[j]) {
				uint32_t hit = (uint32_t)t * 4u + a->start_base_offset - (uint32_t)j;
				if (match_exact(read, a, hit, read_len) > 0) return hit;
			}
	}
	return 0xffffffffu;
}

#define CEQ(c, t) ((c)[0] == (t)[0] && (c)[1] == (t)[1])
#define C2EQ(x, y, u, v) ((CEQ(x, u) && CEQ(y, v)) || (CEQ(x, v) && CEQ(y, u)))
#define DONOR_PART(c) (CEQ(c, "GT") || CEQ(c, "AG") || CEQ(c, "AC") || CEQ(c, "CT"))
/* paired_chars_part, core-junction.c:4366-4374 */
static int paired_part(const char *x, const char *y, int rev)
{
	if (C2EQ(x, y, "GT", "AG") || C2EQ(x, y, "CT", "AC")) {
		if (rev && (CEQ(x, "AG") || CEQ(x, "AC"))) return 1;
		if (!rev && (CEQ(x, "CT") || CEQ(x, "GT"))) return 1;
	}
	return 0;
}

/* read_quality_score, gene-algorithms.c:130-152 */
static float quality_score(const char *q, int rl, int base)
{
	int i, qual = 0, n = 0;
	for (i = 0; i < rl; i++) {
		const int v = q[i] - base;
		if (v > 1) { qual += v; n++; }
	}
	return (float)(qual * 1. / n);
}

/* locate_current_value_index, core.c:2216-2249: the block holding the record, else the block
 * of the final voting run (the thread's value index, restored after every record) */
static const garray *value_index(const svg_genome_arrays *g, uint32_t pos, int rlen)
{
	int b;
	if (g->nblocks < 2) return &g->blk[0];
	for (b = 0; b < g->nblocks; b++) {
		uint32_t begin = g->blk[b].start_base_offset, end = g->blk[b].start_base_offset + g->blk[b].length;
		if ((b == 0 && pos >= begin && pos < end - 1000000u) ||
		    (b > 0 && b < g->nblocks - 1 && pos >= begin + 1000000u && pos < end - 1000000u) ||
		    (b == g->nblocks - 1 && pos >= begin + 1000000u && pos < end))
			return &g->blk[b];
	}
	(void)rlen;
	return &g->blk[g->nblocks - 1];
}

/* locate_gene_position (gene-algorithms.c:441-517 with rl = 0): the contig index of a linear
 * position, or -1 where the reference returns no name (padding, past the contig end) */
static int contig_of(const svg_genome_arrays *g, uint32_t linear)
{
	int lo = 0, hi = (int)g->n_chr, n;
	while (hi > lo + 1) {
		int mid = (lo + hi) / 2;
		if (g->chr_end[mid] > linear) hi = mid; else lo = mid + 1;
	}
	n = lo - 2 > 0 ? lo - 2 : 0;
	for (; n < (int)g->n_chr; n++)
		if (g->chr_end[n] > linear) {
			uint32_t pos = n == 0 ? linear : linear - g->chr_end[n - 1];
			if (linear > g->chr_end[n] + 15u - (uint32_t)g->padding) return -1;
			if ((int)pos < g->padding) return -1;
			return n;
		}
	return -1;
}

/* ------------------------------------------------------------------ event table */
/* ids: event id + 1, 0 = end; cap: the list's room (id_list[0]) -- searches read up to cap entries,
 * a put takes the first 0 among the first cap - 1 */
typedef struct { uint32_t key; uint32_t cap; uint32_t ids[EV_PER_SITE]; } site_t;

struct svg_events {
	svg_event *ev;
	uint64_t n, cap;
	site_t *site;
	uint64_t site_cap, site_used;    /* open addressing, key 0 = empty (coordinate 0 is never put) */
};

int svg_events_create(svg_events **out)
{
	svg_events *t;
	if (!out) { svg_set_error("svg_events_create: NULL argument"); return SVG_E_ARG; }
	t = calloc(1, sizeof *t);
	t->site_cap = 1 << 12;
	t->site = calloc(t->site_cap, sizeof(site_t));
	*out = t;
	return 0;
}

void svg_events_destroy(svg_events *t)
{
	if (!t) return;
	free(t->ev);
	free(t->site);
	free(t);
}

int64_t svg_events_count(const svg_events *t) { return t ? (int64_t)t->n : SVG_E_ARG; }

int svg_events_get(const svg_events *t, svg_event *out)
{
	if (!t || (!out && t->n)) { svg_set_error("svg_events_get: NULL argument"); return SVG_E_ARG; }
	if (t->n) memcpy(out, t->ev, sizeof(svg_event) * t->n);
	return 0;
}

static inline uint64_t site_hash(uint32_t k) { return (k * 0x9E3779B97F4A7C15ull) >> 20; }

static site_t *site_find(const svg_events *t, uint32_t key)
{
	uint64_t m = t->site_cap - 1, i = site_hash(key) & m;
	for (;; i = (i + 1) & m) {
		if (t->site[i].key == key) return &t->site[i];
		if (!t->site[i].key) return NULL;
	}
}

static site_t *site_get(svg_events *t, uint32_t key)
{
	uint64_t m, i;
	if (2 * (t->site_used + 1) > t->site_cap) {
		site_t *old = t->site;
		uint64_t oc = t->site_cap, j;
		t->site_cap *= 2;
		t->site = calloc(t->site_cap, sizeof(site_t));
		for (j = 0; j < oc; j++)
			if (old[j].key) {
				uint64_t k = site_hash(old[j].key) & (t->site_cap - 1);
				while (t->site[k].key) k = (k + 1) & (t->site_cap - 1);
				t->site[k] = old[j];
			}
		free(old);
	}
	m = t->site_cap - 1;
	for (i = site_hash(key) & m;; i = (i + 1) & m) {
		if (t->site[i].key == key) return &t->site[i];
		if (!t->site[i].key) {
			t->site[i].key = key;
			t->site[i].cap = EV_PER_SITE;
			t->site_used++;
			return &t->site[i];
		}
	}
}

/* a fresh zeroed event (reallocate_event_space + memset) */
static uint64_t new_event(svg_events *t)
{
	if (t->n == t->cap) {
		t->cap = t->cap ? t->cap * 2 : 1024;
		t->ev = realloc(t->ev, sizeof(svg_event) * t->cap);
	}
	memset(&t->ev[t->n], 0, sizeof(svg_event));
	return t->n++;
}

/* put_new_event, core-indel.c:1385-1419 */
static void put_event(svg_events *t, uint64_t id)
{
	uint32_t sides[2] = {t->ev[id].small_side, t->ev[id].large_side};
	int s, k;
	for (s = 0; s < 2; s++) {
		site_t *st;
		if (!sides[s]) continue;
		st = site_get(t, sides[s]);
		for (k = 0; k + 1 < (int)st->cap; k++)
			if (!st->ids[k]) { st->ids[k] = (uint32_t)id + 1; st->ids[k + 1] = 0; break; }
	}
}

/* search_event by small side, core-indel.c:1420-1461: ids of the events of the given types
 * whose small side is pos, in list order */
static int search_small(const svg_events *t, uint32_t pos, int types, uint64_t *ids)
{
	const site_t *st;
	int k, n = 0;
	if (pos < 1 || pos > 0xffff0000u) return 0;
	if (!(st = site_find(t, pos))) return 0;
	for (k = 0; k < (int)st->cap && st->ids[k]; k++) {
		const svg_event *e = &t->ev[st->ids[k] - 1];
		if (!(e->event_type & types) || e->small_side != pos) continue;
		ids[n++] = st->ids[k] - 1;
	}
	return n;
}

/* local_add_indel_event, core-indel.c:1498-1569: returns the id of a new event, or -1 when an
 * event of this length at this side existed (its id in *old_id, its support + 1) */
static int64_t add_indel_event(svg_events *t, const char *text, uint32_t left_edge, int indels, int64_t *old_id)
{
	uint64_t ids[EV_PER_SITE], id;
	int k, n = search_small(t, left_edge, SVG_EVENT_INDEL | 16 /* LONG_INDEL */, ids);
	svg_event *e;
	for (k = 0; k < n; k++)
		if (t->ev[ids[k]].indel_length == indels) {
			if (old_id) *old_id = (int64_t)ids[k];
			t->ev[ids[k]].supporting_reads++;
			return -1;
		}
	id = new_event(t);
	e = &t->ev[id];
	if (indels < 0) {
		/* set_insertion_sequence keeps base2int of each inserted base (2 bits); decoded here */
		int i, L = -indels < (int)sizeof e->inserted_bases ? -indels : (int)sizeof e->inserted_bases;
		for (i = 0; i < L; i++) {
			char c = text[i];
			e->inserted_bases[i] = "AGCT"[c < 'G' ? (c == 'A' ? 0 : 2) : (c == 'G' ? 1 : 3)];
		}
		e->inserted_len = (uint8_t)L;
	}
	e->small_side = left_edge;
	e->large_side = left_edge + 1 + (indels > 0 ? indels : 0);
	e->event_type = SVG_EVENT_INDEL;
	e->indel_length = (int16_t)indels;
	e->supporting_reads = 1;
	e->event_quality = 1.0f;
	put_event(t, id);
	return (int64_t)id;
}

/* ------------------------------------------------------------------ per-record searches */
typedef struct {
	int16_t *dp;          /* (rl + 16) x rl score table, row-major */
	uint8_t *mask;
	int rows, cols;
	/* a traceback takes at most rows + len <= 2 * len + 16 steps (the reference sizes its stack
	 * buffer len * 10 / 7, core-indel.c; here the walk also stops at the end of the buffer) */
	char mv[2 * (SVG_MAX_READ_LENGTH + 16) + 64];
} scratch_t;

/* find_subread_end, input-files.c:1371-1387 */
static int subread_end(int len, int total, int subread)
{
	int step;
	if (len <= LONG_READ) {
		step = ((len << 16) - (19 << 16)) / (total - 1);
		return ((step * subread) >> 16) + 15;
	}
	step = 6 << 16;
	if (((len - 18) << 16) / step > 62) step = ((len - 18) << 16) / 62;
	return ((step * subread) >> 16) + 15;
}

/* core_dynamic_align, core-indel.c:4573-4787: banded global alignment of read[0..len) to the
 * genome from begin; movements 0 match, 1 deletion, 2 insertion, 3 mismatch; 0 if the path's
 * net offset is not expected_offset */
static int dynamic_align(scratch_t *s, const garray *a, const svg_event_params *ep, int max_indel_length,
                         const char *read, int len, uint32_t begin, int expected_offset)
{
	const int max_indel = max_indel_length < 16 ? max_indel_length : 16;
	const int rows = len + expected_offset;
	int i, j, out = 0, delta = 0, path_i;
	if (len < 3 || abs(expected_offset) > max_indel) return 0;
	if (expected_offset < 0 && len < 3 - expected_offset) return 0;
#define T(i, j) s->dp[(size_t)(i) * s->cols + (j)]
#define M(i, j) s->mask[(size_t)(i) * s->cols + (j)]
	for (i = 0; i < rows; i++)
		for (j = 0; j < len; j++) {
			int16_t up, left, diag;
			char ch;
			int sc;
			M(i, j) = 0;
			if (j < i - max_indel || j > max_indel + i) { T(i, j) = -9999; continue; }
			up = i > 0 ? (int16_t)(T(i - 1, j) + (M(i - 1, j) == MASK_DELETION ? ep->dp_penalty_extend_gap : ep->dp_penalty_create_gap)) : -9999;
			left = j > 0 ? (int16_t)(T(i, j - 1) + (M(i, j - 1) == MASK_INSERTION ? ep->dp_penalty_extend_gap : ep->dp_penalty_create_gap)) : -9999;
			ch = gv_get(a, begin + i);
			sc = ch == read[j] ? ep->dp_match_score : ep->dp_mismatch_penalty;
			if (i > 0 && j > 0) diag = (int16_t)(T(i - 1, j - 1) + sc);
			else if (i == 0 && j == 0) diag = (int16_t)sc;
			else diag = -9999;
			if (diag == up && diag > left) { M(i, j) = MASK_DELETION; T(i, j) = up; }
			else if (diag == left && diag > up) { M(i, j) = MASK_INSERTION; T(i, j) = left; }
			else if (diag > left && diag > up) { M(i, j) = ch == read[j] ? MASK_MATCH : MASK_MISMATCH; T(i, j) = diag; }
			else if (diag == left && diag == up) { M(i, j) = ch == read[j] ? MASK_MATCH : MASK_MISMATCH; T(i, j) = diag; }
			else if (left > up) { M(i, j) = MASK_INSERTION; T(i, j) = left; }
			else { M(i, j) = MASK_DELETION; T(i, j) = up; }
		}
	path_i = rows - 1;
	j = len - 1;
	for (;;) {
		int m = M(path_i, j);
		if (out >= (int)sizeof s->mv) return 0;
		if (m == MASK_INSERTION) { j--; delta--; s->mv[out++] = 2; }
		else if (m == MASK_DELETION) { path_i--; delta++; s->mv[out++] = 1; }
		else { s->mv[out++] = m == MASK_MATCH ? 0 : 3; path_i--; j--; }
		if (path_i == -1 && j == -1) break;
		if (j < 0 || path_i < 0) return 0;
	}
#undef T
#undef M
	if (expected_offset != delta) return 0;
	for (i = 0; i < out / 2; i++) { char x = s->mv[out - 1 - i]; s->mv[out - 1 - i] = s->mv[i]; s->mv[i] = x; }
	return out;
}

static inline int8_t min_dist(int8_t cur, int dist)
{
	/* connected_*_event_distance: set when < 1, else the smaller (char fields) */
	if (cur < 1) return (int8_t)dist;
	return (int8_t)(dist < cur ? dist : cur);
}

/* find_new_indels, core-indel.c:1831-2098 (dynamic-programming path) */
static void find_indels(svg_events *t, scratch_t *s, const garray *a, const svg_params *p, const svg_event_params *ep,
                        svg_mapping_result *r, const char *text, int rl)
{
	const int16_t *rec = r->selected_indel_record;
	const uint32_t vpos = r->selected_position;
	int i, last_correct_subread = 0, last_indel = 0;
	if (!rec[0]) return;
	for (i = 0; rec[i] && i < MAX_INDEL_SECT; i += 3) {
		const int indels = rec[i + 2] - last_indel;
		const int next_correct_subread = rec[i] - 1;
		if (indels) {
			int last_cb = subread_end(rl, p->total_subreads, last_correct_subread) - 9;
			int first_cb = subread_end(rl, p->total_subreads, next_correct_subread) - 16 + 9;
			int steps, x, total_mm = 0, last_mv = 0, in_indel = 0, cur_len = 0;
			int64_t last_event_id = -1;
			uint32_t chr, left_boundary = 0;
			int cursor_read;
			last_cb = last_cb < 0 ? 0 : last_cb;
			last_cb = last_cb < rl - 1 ? last_cb : rl - 1;
			first_cb = first_cb < rl - 1 ? first_cb : rl - 1;
			first_cb = first_cb > 0 ? first_cb : 0;
			first_cb = first_cb > last_cb ? first_cb : last_cb;
			first_cb = first_cb + 10 < rl ? first_cb + 10 : rl;
			steps = dynamic_align(s, a, ep, p->max_indel_length, text + last_cb, first_cb - last_cb,
			                      vpos + last_cb + last_indel, indels);
			chr = vpos + last_cb + last_indel;
			cursor_read = last_cb;
			for (x = 0; x < steps; x++) total_mm += s->mv[x] == 3;
			if (total_mm <= 2)
				for (x = 0; x < steps; x++) {
					const int mv = s->mv[x];
					if (last_mv != mv) {
						if ((mv == 1 || mv == 2) && !in_indel) {
							left_boundary = chr;
							in_indel = 1;
							cur_len = 0;
						} else if (in_indel && (mv == 0 || mv == 3)) {
							if (abs(cur_len) <= p->max_indel_length) {
								int64_t old_id = -1, nid;
								nid = add_indel_event(t, text + cursor_read + (cur_len < 0 ? cur_len : 0), left_boundary - 1,
								                      cur_len, &old_id);
								r->result_flags |= GAPPED_FLAG;
								if (last_event_id >= 0) {
									svg_event *last = &t->ev[last_event_id], *cur = &t->ev[nid >= 0 ? nid : old_id];
									const int dist = (int)(left_boundary - last->large_side);
									last->connected_next_event_distance = min_dist(last->connected_next_event_distance, dist);
									cur->connected_previous_event_distance = min_dist(cur->connected_previous_event_distance, dist);
								}
								last_event_id = nid >= 0 ? nid : old_id;
							}
						}
						if (mv == 0 || mv == 3) in_indel = 0;
					}
					if (in_indel && mv == 1) cur_len++;
					if (in_indel && mv == 2) cur_len--;
					if (mv == 1 || mv == 3 || mv == 0) chr++;
					if (mv == 2 || mv == 3 || mv == 0) cursor_read++;
					last_mv = mv;
				}
		}
		last_correct_subread = rec[i + 1] - 1;
		last_indel = rec[i + 2];
	}
}

/* a junction event at (small, large): another read for an existing one (any event type of the
 * search) or a new junction (core-junction.c:4522-4566, 5372-5414) */
static void add_junction_event(svg_events *t, uint32_t small, uint32_t large, int gtag)
{
	uint64_t ids[EV_PER_SITE], id;
	int k, n = search_small(t, small, SVG_EVENT_JUNCTION | SVG_EVENT_FUSION, ids);
	svg_event *e;
	for (k = 0; k < n; k++)
		if (t->ev[ids[k]].large_side == large) { t->ev[ids[k]].supporting_reads++; return; }
	id = new_event(t);
	e = &t->ev[id];
	e->small_side = small;
	e->large_side = large;
	e->is_negative_strand = (int8_t)!gtag;
	e->event_type = SVG_EVENT_JUNCTION;
	e->supporting_reads = 1;
	put_event(t, id);
}

/*
 * The events of one fragile-voting window (core_fragile_junction_voting, core-junction.c:5211-5419):
 * every reported top-vote slot's recorder sections go through core_dynamic_align on the window
 * text (in, wl bases, NUL-terminated) and its movement walk; then the window's junction.
 */
static void fragile_window_events(svg_events *t, scratch_t *s, const garray *a, const svg_params *p,
                                  const svg_event_params *ep, int gap, const svg_fragile_window *W,
                                  const svg_fragile_slot *slots, const char *in)
{
	const int wl = W->length;
	uint32_t q;
	for (q = 0; q < W->n_slots; q++) {
		const svg_fragile_slot *S = &slots[W->first_slot + q];
		const int16_t *rec = S->rec;
		int kk, last_correct_subread = 0;
		for (kk = 0; kk < MAX_INDEL_SECT && rec[kk]; kk += 3) {
			const int indels = rec[kk + 2];   /* last_indel stays 0 in the reference's loop */
			int last_cb, first_cb, steps, x, total_mm = 0, last_mv = 0, in_indel = 0, cur_len = 0, cursor_read;
			int64_t last_event_id = -1;
			uint32_t chr, left_boundary = 0;
			if (!indels) continue;
			last_cb = subread_end(wl, p->total_subreads, last_correct_subread) - 9;
			first_cb = subread_end(wl, p->total_subreads, rec[kk] - 1) - 16 + 9;
			first_cb = first_cb + 10 < wl ? first_cb + 10 : wl;
			last_cb = last_cb > 0 ? last_cb : 0;
			last_cb = last_cb < wl - 1 ? last_cb : wl - 1;
			steps = dynamic_align(s, a, ep, p->max_indel_length, in + last_cb, first_cb - last_cb, S->position + (uint32_t)last_cb,
			                      indels);
			chr = S->position + (uint32_t)last_cb;
			cursor_read = last_cb;
			for (x = 0; x < steps; x++) total_mm += s->mv[x] == 3;
			if (total_mm < 2 || (ep->maximise_sensitivity_indel && total_mm <= 2))
				for (x = 0; x < steps; x++) {
					const int mv = s->mv[x];
					if (last_mv != mv) {
						if ((mv == 1 || mv == 2) && !in_indel) {
							left_boundary = chr;
							in_indel = 1;
							cur_len = 0;
						} else if (in_indel && (mv == 0 || mv == 3)) {
							/* (the ambiguity count the reference computes here is not used) */
							if (abs(cur_len) <= p->max_indel_length) {
								int64_t nid = add_indel_event(t, in + cursor_read + (cur_len < 0 ? cur_len : 0), left_boundary - 1,
								                              cur_len, NULL);
								if (last_event_id >= 0 && nid >= 0) {
									svg_event *last = &t->ev[last_event_id], *cur = &t->ev[nid];
									const int dist = (int)(cur->small_side - last->large_side + 1);
									cur->connected_previous_event_distance = (int8_t)dist;
									last->connected_next_event_distance = (int8_t)dist;
								}
								last_event_id = nid;
							}
						}
						if (mv == 0 || mv == 3) in_indel = 0;
					}
					if (in_indel && mv == 1) cur_len++;
					if (in_indel && mv == 2) cur_len--;
					if (mv == 1 || mv == 3 || mv == 0) chr++;
					if (mv == 2 || mv == 3 || mv == 0) cursor_read++;
					last_mv = mv;
				}
			/* the reference reads indel_recorder[i + 1] with the voting loop's i (== gap) here */
			last_correct_subread = rec[gap + 1] - 1;
		}
	}
	if (W->junction) add_junction_event(t, W->small_side, W->large_side, W->gtag);
}

#define SE_MIN 18        /* SHORT_EXON_MIN_LENGTH, core-junction.c:4381 */
#define SE_WINDOW 6      /* SHORT_EXON_WINDOW */
#define SE_EXTEND 5000u  /* SHORT_EXON_EXTEND */

/* core_search_short_exons, core-junction.c:4386-4731 (reads > 160 bp): a short exon before the
 * head or after the tail of the record's coverage, found by an exact 7-base search within 5 kbp
 * and a GT..AG / CT..AC donor pair, becomes a junction event */
static void short_exons(svg_events *t, const garray *a, const svg_event_params *ep, const char *read_text, const char *qual,
                        int rl, uint32_t p1, uint32_t p2, int cov_start, int cov_end)
{
	const char *inb = read_text;
	const uint32_t pos_small = p1 < p2 ? p1 : p2, pos_big = p1 < p2 ? p2 : p1;
	uint32_t best_j1 = 0, best_j2 = 0;
	int need_to_test = 0, max_score, max_gtag = 0;
	/* the head */
	if (cov_start > SE_MIN) {
		int need_check2 = 1;
		if (qual && qual[0] && quality_score(qual, SE_MIN, ep->quality_base) < 6) need_check2 = 0;
		if (need_check2 && SE_MIN * 0.6 < match_chro(inb, a, pos_small, SE_MIN)) need_check2 = 0;
		if (need_check2) {
			int d, is_indel = 0, tp;
			for (d = -3; d <= 3; d++)
				if (match_chro(inb, a, pos_small + (uint32_t)d, SE_MIN) >= SE_MIN * .7) { is_indel = 1; break; }
			if (!is_indel)
				for (tp = SE_MIN; tp < cov_start; tp++) {
					char cc[2];
					chro_2base(a, pos_small + (uint32_t)tp, 0, cc);
					if (DONOR_PART(cc)) { need_to_test = 1; break; }
				}
		}
	}
	max_score = -999;
	if (need_to_test && pos_small >= SE_MIN) {
		uint32_t test_end = pos_small - SE_EXTEND, new_pos = pos_small - SE_MIN;
		if (SE_EXTEND > pos_small) test_end = 0;
		for (;;) {
			int sp;
			new_pos = match_chro_range(inb, a, new_pos, 7, new_pos - test_end, 1);
			if (new_pos == 0xffffffffu) break;
			for (sp = SE_MIN; sp < cov_start; sp++) {
				char cc[2], cc2[2];
				chro_2base(a, pos_small + (uint32_t)sp - 2, 0, cc);
				if (!DONOR_PART(cc)) continue;
				chro_2base(a, new_pos + (uint32_t)sp, 0, cc2);
				if (DONOR_PART(cc2) && paired_part(cc2, cc, 0)) {
					const int m_old = match_chro(inb + sp, a, pos_small + (uint32_t)sp, SE_WINDOW);
					const int m_new = match_chro(inb, a, new_pos, sp);
					const int score = (int)(1000000u + (uint32_t)(m_new * 10000) + (uint32_t)(m_old * 1000) + new_pos - test_end);
					if (score <= max_score) continue;
					max_score = score;
					if (m_new < sp || m_old < SE_WINDOW) continue;
					max_gtag = cc2[0] == 'G' || cc2[1] == 'G';
					best_j1 = new_pos + (uint32_t)sp - 1;
					best_j2 = pos_small + (uint32_t)sp;
				}
			}
		}
	}
	if (best_j1 > 0) add_junction_event(t, best_j1, best_j2, max_gtag);
	/* the tail */
	need_to_test = 0;
	max_score = -999;
	if (cov_end < rl - SE_MIN) {
		int need_check2 = 1;
		if (qual && qual[0] && quality_score(qual + rl - SE_MIN, SE_MIN, ep->quality_base) < 6) need_check2 = 0;
		if (SE_MIN * 0.6 < match_chro(inb + rl - SE_MIN, a, pos_big + (uint32_t)(rl - SE_MIN), SE_MIN)) need_check2 = 0;
		if (need_check2) {
			int d, is_indel = 0, tp;
			for (d = -3; d <= 3; d++)
				if (match_chro(inb + rl - SE_MIN, a, pos_big + (uint32_t)(rl - SE_MIN) + (uint32_t)d, SE_MIN) >= SE_MIN * .7) {
					is_indel = 1;
					break;
				}
			if (!is_indel)
				for (tp = cov_end; tp < rl; tp++) {
					char cc[2];
					chro_2base(a, pos_big + (uint32_t)tp, 0, cc);
					if (DONOR_PART(cc)) { need_to_test = 1; break; }
				}
		}
	}
	best_j1 = 0;
	max_gtag = 0;
	if (need_to_test) {
		uint32_t test_end = pos_big + SE_EXTEND, new_pos = pos_big + (uint32_t)rl - SE_MIN + 16;
		if (test_end > a->length + a->start_point) test_end = a->length + a->start_point;
		for (;;) {
			int sp;
			if (new_pos + test_end - new_pos < a->start_base_offset + a->length)
				new_pos = match_chro_range(inb + rl - SE_MIN, a, new_pos, 7, test_end - new_pos, 0);
			else break;
			if (new_pos == 0xffffffffu) break;
			for (sp = cov_end; sp < rl - SE_MIN; sp++) {
				char cc[2], cc2[2];
				const uint32_t tail = new_pos + SE_MIN - (uint32_t)rl + (uint32_t)sp;
				chro_2base(a, pos_big + (uint32_t)sp, 0, cc);
				if (!DONOR_PART(cc)) continue;
				chro_2base(a, tail - 2, 0, cc2);
				if (DONOR_PART(cc2) && paired_part(cc, cc2, 0)) {
					const int m_new = match_chro(inb + sp, a, tail, rl - sp);
					const int m_old = match_chro(inb + sp - SE_WINDOW, a, pos_big + (uint32_t)sp - SE_WINDOW, SE_WINDOW);
					const int score = (int)(1000000u + (uint32_t)(m_new * 10000) + (uint32_t)(m_old * 1000) + test_end - new_pos);
					if (score <= max_score) continue;
					max_score = score;
					if (m_new < rl - sp || m_old < SE_WINDOW) continue;
					max_gtag = cc[0] == 'G' || cc[1] == 'G';
					best_j1 = pos_big + (uint32_t)sp - 1;
					best_j2 = tail;
				}
			}
		}
	}
	if (best_j1 > 0) add_junction_event(t, best_j1, best_j2, max_gtag);
}

/* is_ambiguous_voting, core-junction.c:3522-3566 */
static int ambiguous_voting(const svg_params *p, const uint16_t *bm, int vote, int max_start, int max_end, int rl, int neg)
{
	int k, enc = 0;
	if (p->big_margin_record_size < 3) return 0;
	if (neg) { int x = max_start; max_start = rl - max_end; max_end = rl - x; }
	for (k = 0; k < p->big_margin_record_size / 3; k++) {
		if (!bm[k * 3]) break;
		if (bm[k * 3] >= vote - 1) {
			if (vote >= bm[k * 3]) { if (bm[k * 3 + 1] >= max_start - 4 && bm[k * 3 + 2] <= max_end + 4) enc++; }
			else if (bm[k * 3 + 1] <= max_start + 4 && bm[k * 3 + 2] >= max_end - 4) enc++;
		}
	}
	return enc > 1 ? enc : 0;
}

/* find_new_junctions, core-junction.c:3836-4137, reads <= 160 bp, no fusion detection */
static void find_junctions(svg_events *t, const svg_genome_arrays *g, const svg_params *p, svg_mapping_result *r,
                           const svg_subjunc_result *j, const uint16_t *bm, int rl, uint64_t read_no, int end)
{
	const int split = j->split_point;
	uint32_t left_vh, right_vh, left_edge, right_edge;
	int gtag, donor_found, jumped, cl, cr;
	if (j->minor_votes < 1) return;
	if (p->do_big_margin_filtering_for_junctions &&
	    ambiguous_voting(p, bm, r->selected_votes, r->confident_coverage_start, r->confident_coverage_end, rl,
	                     (r->result_flags & NEG_FLAG) ? 1 : 0))
		return;
	left_vh = r->selected_position < j->minor_position ? r->selected_position : j->minor_position;
	right_vh = r->selected_position > j->minor_position ? r->selected_position : j->minor_position;
	gtag = r->result_flags & 3;
	donor_found = gtag < 3;
	jumped = (r->result_flags & JUMPED_FLAG) ? 1 : 0;
	if (split <= 0) return;
	if (jumped) {
		uint32_t major_small = r->selected_position + split, minor_small = j->minor_position + rl - split;
		int abnormal = (j->minor_coverage_start > r->confident_coverage_start) + (minor_small > major_small) == 1;
		int small_neg = ((r->result_flags & NEG_FLAG) ? 1 : 0) + (minor_small < major_small) == 1;
		left_edge = major_small < minor_small ? major_small : minor_small;
		right_edge = major_small > minor_small ? major_small : minor_small;
		if (!(r->result_flags & NEG_FLAG)) abnormal = !abnormal;
		if (small_neg != abnormal) { left_edge--; right_edge--; }
	} else {
		int sl = split, sr = split, minor_off = j->double_indel_offset & 0xf, major_off = (j->double_indel_offset >> 4) & 0xf;
		if ((j->minor_coverage_start > r->confident_coverage_start) + (j->minor_position > r->selected_position) == 1) sr--;
		else sl--;
		if (major_off >= 8) major_off = -(16 - major_off);
		left_edge = left_vh + sl + (r->selected_position > j->minor_position ? minor_off : major_off);
		right_edge = right_vh + sr;
	}
	cl = contig_of(g, left_edge);
	cr = contig_of(g, right_edge);
	if (cl != cr) return;
	{
		uint64_t ids[EV_PER_SITE], id;
		int k, n = search_small(t, left_edge, SVG_EVENT_INDEL | SVG_EVENT_JUNCTION | SVG_EVENT_FUSION, ids);
		int64_t found = -1;
		int type;
		svg_event *e;
		for (k = 0; k < n; k++)
			if (t->ev[ids[k]].large_side == right_edge) { found = (int64_t)ids[k]; break; }
		r->result_flags |= GAPPED_FLAG;
		if (found >= 0) { t->ev[found].supporting_reads++; return; }
		id = new_event(t);
		e = &t->ev[id];
		e->small_side = left_edge;
		e->large_side = right_edge + j->indel_at_junction;
		e->critical_read_id = 2ull * read_no + (uint64_t)end;
		type = SVG_EVENT_JUNCTION;
		if (jumped) type = SVG_EVENT_FUSION;
		if ((j->minor_coverage_start > r->confident_coverage_start) + (j->minor_position > r->selected_position) == 1)
			type = SVG_EVENT_FUSION;
		if (right_edge - left_edge > (uint32_t)p->maximum_intron_length) type = 0;
		{
			const uint32_t dist = e->large_side - e->small_side;
			if (dist > MAX_INSERTION && type == SVG_EVENT_FUSION) {
				int cov_end = j->minor_coverage_end > r->confident_coverage_end ? j->minor_coverage_end : r->confident_coverage_end;
				int cov_start = j->minor_coverage_start < r->confident_coverage_start ? j->minor_coverage_start : r->confident_coverage_start;
				int major_cov = r->confident_coverage_end - r->confident_coverage_start;
				if (cov_end - cov_start < rl - 15 || major_cov > rl - 15) type = 0;
			}
			if (dist > MAX_INSERTION && type == SVG_EVENT_FUSION && j->minor_votes < 2) type = 0;
			else if (type == SVG_EVENT_FUSION && j->minor_votes < 1) type = 0;
			if (dist > MAX_INSERTION && type == SVG_EVENT_FUSION && r->selected_votes < 2) type = 0;
			else if (type == SVG_EVENT_FUSION && r->selected_votes < 1) type = 0;
			if (dist > MAX_INSERTION && type == SVG_EVENT_FUSION && (split < rl * 0.2 || split >= rl * 0.8)) type = 0;
		}
		if (type == SVG_EVENT_JUNCTION) {
			e->is_negative_strand = !gtag;
			e->event_type = SVG_EVENT_JUNCTION;
			e->supporting_reads = 1;
			e->indel_at_junction = j->indel_at_junction;
			e->is_donor_found_or_annotation = (int8_t)donor_found;
			e->small_side_increasing_coordinate = j->small_side_increasing_coordinate;
			e->large_side_increasing_coordinate = j->large_side_increasing_coordinate;
			put_event(t, id);
		}
		/* fusions are recorded only with fusion / long-deletion detection: the slot stays
		 * type 0 (CHRO_EVENT_TYPE_REMOVED) like the reference's */
	}
}

/* reverse_read (input-files.c:1113-1189, base space) with its conversion table: A/C/G/T/U
 * complemented, every other character -> 'N' */
static inline char rc_char(char c)
{
	switch (c) { case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A'; case 'U': return 'A'; }
	return 'N';
}
static void reverse_read(char *s, int len)
{
	int i;
	for (i = 0; i < len / 2; i++) { char x = s[len - 1 - i]; s[len - 1 - i] = rc_char(s[i]); s[i] = rc_char(x); }
	if (i * 2 == len - 1) s[i] = rc_char(s[i]);
}

/* has_better_mapping, core.c:3035-3047 (unsigned position arithmetic as in the reference) */
static int has_better_mapping(const svg_params *p, const svg_mapping_result *recs, int b)
{
	const svg_mapping_result *x = &recs[b];
	int k;
	for (k = 0; k < b; k++) {
		const svg_mapping_result *y = &recs[k];
		if (x->selected_position >= y->selected_position - (uint32_t)p->max_indel_length - 1u &&
		    x->selected_position <= y->selected_position + (uint32_t)p->max_indel_length + 1u)
			if (x->confident_coverage_start >= y->confident_coverage_start &&
			    x->confident_coverage_end <= y->confident_coverage_end) return 1;
	}
	return 0;
}

static void reverse_chars(char *s, int len)
{
	int i;
	for (i = 0; i < len / 2; i++) { char x = s[i]; s[i] = s[len - 1 - i]; s[len - 1 - i] = x; }
}

/* the strand-s text of an end as do_voting sees it (-S reversal at fetch, then reverse_read for
 * strand 1), NUL-terminated */
static int strand_text(const svg_params *p, const svg_reads *rr, int e, uint64_t i, int strand, char *text)
{
	int rl = rr->lens[i];
	if (rl > SVG_READ_KEEP) rl = SVG_READ_KEEP;
	memcpy(text, rr->seq + rr->offsets[i], (size_t)rl);
	text[rl] = 0;
	if (e ? p->reverse_r2 : p->reverse_r1) reverse_read(text, rl);
	if (strand) reverse_read(text, rl);
	return rl;
}

/* the events of every window [*w, ...) of block `blk` and read `read` (or of every read when
 * read == UINT64_MAX), in the windows' order */
static void fragile_events(svg_events *t, scratch_t *s, const svg_genome_arrays *g, const svg_params *p,
                           const svg_event_params *ep, const svg_reads *r1, const svg_reads *r2, const svg_fragile_result *fr,
                           uint64_t *w, int blk, uint64_t read)
{
	char text[SVG_MAX_READ_LENGTH + 2];
	uint64_t cur = UINT64_MAX;
	int cur_key = -1;
	while (*w < fr->n_windows) {
		const svg_fragile_window *W = &fr->windows[*w];
		const int key = W->strand * 2 + W->end;
		char in[SVG_MAX_READ_LENGTH + 2];
		if (W->block != blk || (read != UINT64_MAX && W->read != read)) break;
		if (W->read != cur || key != cur_key) {
			strand_text(p, W->end ? r2 : r1, W->end, W->read, W->strand, text);
			cur = W->read;
			cur_key = key;
		}
		memcpy(in, text + W->start, W->length);
		in[W->length] = 0;
		fragile_window_events(t, s, &g->blk[blk], p, ep, g->gap, W, fr->slots, in);
		(*w)++;
	}
}

int svg_events_add_batch2(svg_events *t, const svg_genome_arrays *g, const svg_params *p, const svg_event_params *ep_in,
                          const svg_reads *r1, const svg_reads *r2, const svg_reads *q1, const svg_reads *q2,
                          uint64_t first_read, svg_mapping_result *out, const svg_subjunc_result *jout,
                          const uint16_t *big_margin, const svg_fragile_result *fr)
{
	const int ends = r2 ? 2 : 1, mb = p ? p->multi_best : 0;
	svg_event_params epd;
	const svg_event_params *ep = ep_in;
	scratch_t *s;
	uint64_t i, w = 0;
	int long_reads = 0;
	if (!t || !g || !p || !r1 || !out) { svg_set_error("svg_events_add_batch: NULL argument"); return SVG_E_ARG; }
	if (r2 && r2->n_reads != r1->n_reads) { svg_set_error("svg_events_add_batch: r1/r2 differ in length"); return SVG_E_ARG; }
	if (mb < 1 || mb > 3 || p->total_subreads < 2) { svg_set_error("svg_events_add_batch: bad parameters"); return SVG_E_ARG; }
	if (p->do_breakpoint_detection && !jout) { svg_set_error("svg_events_add_batch: subjunc records required"); return SVG_E_ARG; }
	if (p->do_breakpoint_detection && p->do_big_margin_filtering_for_junctions && !big_margin) {
		svg_set_error("svg_events_add_batch: big-margin records required"); return SVG_E_ARG;
	}
	if (!ep) { svg_event_params_default(&epd); ep = &epd; }
	if (p->do_breakpoint_detection)
		for (i = 0; i < r1->n_reads && !long_reads; i++)
			if (r1->lens[i] > LONG_READ || (r2 && r2->lens[i] > LONG_READ)) long_reads = 1;
	if (long_reads && !fr) {
		svg_set_error("subjunc reads over %d bp need their fragile junction votes (svg_fragile_batch, svg_events_add_batch2)",
		              LONG_READ);
		return SVG_E_UNSUPPORTED;
	}
	if (fr) {
		for (i = 0; i < fr->n_windows; i++)
			if (fr->windows[i].block >= g->nblocks || fr->windows[i].read >= r1->n_reads ||
			    (fr->windows[i].end && !r2) || fr->windows[i].first_slot + fr->windows[i].n_slots > fr->n_slots) {
				svg_set_error("svg_events_add_batch2: fragile windows do not match the batch / index");
				return SVG_E_ARG;
			}
	}
	s = calloc(1, sizeof *s);
	s->cols = SVG_MAX_READ_LENGTH;
	s->rows = SVG_MAX_READ_LENGTH + 20;
	s->dp = malloc(sizeof(int16_t) * (size_t)s->rows * s->cols);
	s->mask = malloc((size_t)s->rows * s->cols);
	if (!s->dp || !s->mask) { free(s->dp); free(s->mask); free(s); svg_set_error("out of memory"); return SVG_E_NOMEM; }
	/* the earlier runs of the block loop: every read's fragile windows, block by block */
	if (fr)
		for (int b = 0; b + 1 < g->nblocks; b++) fragile_events(t, s, g, p, ep, r1, r2, fr, &w, b, UINT64_MAX);
	for (i = 0; i < r1->n_reads; i++) {
		int e;
		/* the final run: this read's windows of the last block, then its tail (core.c:3240-3290) */
		if (fr) fragile_events(t, s, g, p, ep, r1, r2, fr, &w, g->nblocks - 1, i);
		for (e = 0; e < ends; e++) {
			const svg_reads *rr = e ? r2 : r1, *qq = e ? q2 : q1;
			char text[SVG_MAX_READ_LENGTH + 2], qual[SVG_MAX_READ_LENGTH + 2];
			int rl = rr->lens[i], b, has_reversed;
			svg_mapping_result *recs = out + ((size_t)i * ends + e) * mb;
			if (rl > SVG_READ_KEEP) rl = SVG_READ_KEEP;
			memcpy(text, rr->seq + rr->offsets[i], (size_t)rl);
			text[rl] = 0;
			qual[0] = 0;
			if (qq) {
				memcpy(qual, qq->seq + qq->offsets[i], (size_t)rl);
				qual[rl] = 0;
			}
			/* -S reversal at fetch (core.c:1186-1198: text and quality), then the strand loop's one
			 * reversal of the text after strand 0 (core.c:3229-3234); the tail reverses text and
			 * quality together, so they stay in opposite orientations */
			if (e ? p->reverse_r2 : p->reverse_r1) { reverse_read(text, rl); if (qq) reverse_chars(qual, rl); }
			reverse_read(text, rl);
			has_reversed = 1;
			for (b = 0; b < mb; b++) {
				svg_mapping_result *r = &recs[b];
				const garray *a;
				int should;
				if (r->selected_votes < 1) continue;
				should = (r->result_flags & NEG_FLAG) ? 1 : 0;
				if (should != has_reversed) {
					has_reversed = !has_reversed;
					reverse_read(text, rl);
					if (qq) reverse_chars(qual, rl);
				}
				a = value_index(g, r->selected_position, rl);
				if (!has_better_mapping(p, recs, b)) find_indels(t, s, a, p, ep, r, text, rl);
				if (p->do_breakpoint_detection) {
					const svg_subjunc_result *j = &jout[((size_t)i * ends + e) * mb + b];
					if (rl > LONG_READ)
						short_exons(t, a, ep, text, qq ? qual : "", rl, r->selected_position,
						            j->minor_votes < 1 ? r->selected_position : j->minor_position, r->confident_coverage_start,
						            r->confident_coverage_end);
					find_junctions(t, g, p, r, j, big_margin ? big_margin + ((size_t)i * ends + e) * SVG_BIG_MARGIN_WORDS : NULL,
					               rl, first_read + i, e);
				}
			}
		}
	}
	free(s->dp); free(s->mask); free(s);
	return 0;
}

int svg_events_add_windows(svg_events *t, const svg_genome_arrays *g, const svg_params *p, const svg_event_params *ep_in,
                           const svg_reads *r1, const svg_reads *r2, const svg_fragile_result *fr, int block)
{
	svg_event_params epd;
	const svg_event_params *ep = ep_in;
	if (!t || !g || !p || !r1 || !fr) { svg_set_error("svg_events_add_windows: NULL argument"); return SVG_E_ARG; }
	if (block < 0 || block >= g->nblocks) { svg_set_error("svg_events_add_windows: block %d of %d", block, g->nblocks); return SVG_E_ARG; }
	for (uint64_t i = 0; i < fr->n_windows; i++)
		if (fr->windows[i].block != (uint32_t)block || fr->windows[i].read >= r1->n_reads || (fr->windows[i].end && !r2) ||
		    fr->windows[i].first_slot + fr->windows[i].n_slots > fr->n_slots) {
			svg_set_error("svg_events_add_windows: fragile windows do not match the batch / block");
			return SVG_E_ARG;
		}
	if (!ep) { svg_event_params_default(&epd); ep = &epd; }
	scratch_t *s = calloc(1, sizeof *s);
	if (!s) { svg_set_error("out of memory"); return SVG_E_NOMEM; }
	s->cols = SVG_MAX_READ_LENGTH;
	s->rows = SVG_MAX_READ_LENGTH + 20;
	s->dp = malloc(sizeof(int16_t) * (size_t)s->rows * s->cols);
	s->mask = malloc((size_t)s->rows * s->cols);
	if (!s->dp || !s->mask) { free(s->dp); free(s->mask); free(s); svg_set_error("out of memory"); return SVG_E_NOMEM; }
	uint64_t w = 0;
	fragile_events(t, s, g, p, ep, r1, r2, fr, &w, block, UINT64_MAX);
	free(s->dp); free(s->mask); free(s);
	return 0;
}

int svg_events_add_batch(svg_events *t, const svg_genome_arrays *g, const svg_params *p, const svg_event_params *ep,
                         const svg_reads *r1, const svg_reads *r2, uint64_t first_read, svg_mapping_result *out,
                         const svg_subjunc_result *jout, const uint16_t *big_margin)
{
	return svg_events_add_batch2(t, g, p, ep, r1, r2, NULL, NULL, first_read, out, jout, big_margin, NULL);
}

/* ------------------------------------------------------------------ merge (finalise) */
typedef struct { const svg_event *e; uint64_t order; } mref_t;

/* conc_sort_compare, core-indel.c:944-970 (|value| 2-3: different events, 0-1: same event) */
static int conc_compare(const svg_event *l, const svg_event *r)
{
	if (l->small_side > r->small_side) return 3;
	if (l->small_side < r->small_side) return -3;
	if (l->large_side > r->large_side) return 3;
	if (l->large_side < r->large_side) return -3;
	if (abs(l->indel_length) < abs(r->indel_length)) return 2;
	if (abs(l->indel_length) > abs(r->indel_length)) return -2;
	if (l->indel_length > r->indel_length) return -2;
	if (l->indel_length < r->indel_length) return 2;
	if ((l->is_donor_found_or_annotation & 64) && !(r->is_donor_found_or_annotation & 64)) return 1;
	if (!(l->is_donor_found_or_annotation & 64) && (r->is_donor_found_or_annotation & 64)) return -1;
	if (l->supporting_reads > r->supporting_reads) return -1;
	if (l->supporting_reads < r->supporting_reads) return 1;
	return 0;
}

static int mref_cmp(const void *a, const void *b)
{
	const mref_t *x = a, *y = b;
	int c = conc_compare(x->e, y->e);
	if (c) return c;
	return x->order < y->order ? -1 : x->order > y->order;
}

int svg_events_merge(svg_events *dst, svg_events *const *tables, int n)
{
	uint64_t total = 0, i, k = 0, start;
	mref_t *refs;
	int ti;
	if (!dst || (n > 0 && !tables)) { svg_set_error("svg_events_merge: NULL argument"); return SVG_E_ARG; }
	for (ti = 0; ti < n; ti++)
		if (!tables[ti] || tables[ti] == dst) { svg_set_error("svg_events_merge: NULL table or dst among the inputs"); return SVG_E_ARG; }
	for (ti = 0; ti < n; ti++) total += tables[ti]->n;
	refs = malloc(sizeof(mref_t) * (total + 1));
	for (ti = 0; ti < n; ti++)
		for (i = 0; i < tables[ti]->n; i++)
			if (tables[ti]->ev[i].event_type) { refs[k].e = &tables[ti]->ev[i]; refs[k].order = k; k++; }
	qsort(refs, k, sizeof(mref_t), mref_cmp);
	/* a group of records of one event: the merged body is a copy of the group's last record
	 * plus the sums / maxima of the others (core-indel.c:1058-1111) */
	for (start = 0; start < k;) {
		uint64_t end = start + 1, m;
		svg_event body;
		while (end < k && abs(conc_compare(refs[end - 1].e, refs[end].e)) <= 1) end++;
		body = *refs[end - 1].e;
		for (m = start; m + 1 < end; m++) {
			const svg_event *o = refs[m].e;
			body.supporting_reads += o->supporting_reads;
			body.anti_supporting_reads += o->anti_supporting_reads;
			body.final_counted_reads += o->final_counted_reads;
			body.final_reads_mismatches += o->final_reads_mismatches;
			body.critical_supporting_reads += o->critical_supporting_reads;
			if (o->junction_flanking_left > body.junction_flanking_left) body.junction_flanking_left = o->junction_flanking_left;
			if (o->junction_flanking_right > body.junction_flanking_right) body.junction_flanking_right = o->junction_flanking_right;
			body.is_donor_found_or_annotation |= o->is_donor_found_or_annotation;
			if (body.connected_next_event_distance > 0 && o->connected_next_event_distance > 0)
				body.connected_next_event_distance = body.connected_next_event_distance < o->connected_next_event_distance ?
				                                     body.connected_next_event_distance : o->connected_next_event_distance;
			else if (o->connected_next_event_distance > body.connected_next_event_distance)
				body.connected_next_event_distance = o->connected_next_event_distance;
			if (body.connected_previous_event_distance > 0 && o->connected_previous_event_distance > 0)
				body.connected_previous_event_distance = body.connected_previous_event_distance < o->connected_previous_event_distance ?
				                                         body.connected_previous_event_distance : o->connected_previous_event_distance;
			else if (o->connected_previous_event_distance > body.connected_previous_event_distance)
				body.connected_previous_event_distance = o->connected_previous_event_distance;
		}
		{
			uint64_t id = new_event(dst);
			dst->ev[id] = body;
			put_event(dst, id);
		}
		start = end;
	}
	free(refs);
	return 0;
}

/* ------------------------------------------------------------------ anti-supporting reads */
typedef struct { uint32_t pos; uint32_t id; } side_t;

static int side_cmp(const void *a, const void *b)
{
	const side_t *x = a, *y = b;
	if (x->pos != y->pos) return x->pos < y->pos ? -1 : 1;
	return x->id < y->id ? -1 : x->id > y->id;
}

/* BINsearch_event, core-indel.c:132-157: an index of pos, else the last index below it (-1) */
static int64_t side_search(const side_t *v, int64_t n, uint32_t pos)
{
	int64_t lo = 0, hi = n - 1;
	for (;;) {
		const int64_t mid = (lo + hi) / 2;
		if (v[mid].pos == pos) return mid;
		if (v[mid].pos < pos) lo = mid + 1; else hi = mid - 1;
		if (lo > hi) return hi;
	}
}

#define ANTI_LIMIT 100   /* ANTI_SUPPORTING_READ_LIMIT, core-indel.c:241 */

/*
 * anti_supporting_read_scan, core-indel.c:177-330, over a (merged) event table: every record
 * with votes (>= min_votes_first; a record with no votes ends the read's list) counts against
 * each event whose small or large side lies strictly inside its covered range shrunk by 5 bases
 * at both ends (an event once per record; at most 100 small-side events per record).
 */
typedef struct {
	const side_t *sm, *lg;
	int64_t ne;
	const svg_params *p;
	const svg_event_params *ep;
	const svg_mapping_result *out;
	uint64_t r0, r1;
	int ends, mb;
	uint32_t *cnt;
} anti_job;

/* anti_supporting_read_scan's per-record body over reads [r0, r1) into the job's counters */
static void *anti_worker(void *arg)
{
	anti_job *J = arg;
	const side_t *sm = J->sm, *lg = J->lg;
	const int64_t ne = J->ne;
	for (uint64_t r = J->r0; r < J->r1; r++) {
		int e, b;
		for (e = 0; e < J->ends; e++)
			for (b = 0; b < J->mb; b++) {
				const svg_mapping_result *m = &J->out[(r * (uint64_t)J->ends + (uint64_t)e) * (uint64_t)J->mb + (uint64_t)b];
				uint32_t cancelled[ANTI_LIMIT];
				int nc = 0;
				int64_t x, l0, l1, r0, r1;
				uint32_t cs, ce;
				if (m->selected_votes < 1) break;
				if (!J->ep->report_multi_mapping_reads && (m->result_flags & 32)) continue;   /* CORE_IS_BREAKEVEN */
				if (m->selected_votes < J->p->min_votes_first) continue;
				cs = m->selected_position + m->confident_coverage_start;
				ce = m->selected_position + m->confident_coverage_end;
				l0 = side_search(sm, ne, cs - 1) + 1;
				l1 = side_search(lg, ne, cs - 1) + 1;
				r0 = side_search(sm, ne, ce) + 20;
				r1 = side_search(lg, ne, ce) + 20;
				for (x = l0; x <= r0 && x < ne && nc < ANTI_LIMIT; x++) {
					const uint32_t pos = sm[x].pos;
					if (pos <= cs + 5 || pos >= ce - 5) continue;
					J->cnt[sm[x].id]++;
					cancelled[nc++] = sm[x].id;
				}
				for (x = l1; x <= r1 && x < ne; x++) {
					const uint32_t pos = lg[x].pos;
					int k, dup = 0;
					if (pos <= cs + 5 || pos >= ce - 5) continue;
					for (k = 0; k < nc; k++) if (cancelled[k] == lg[x].id) { dup = 1; break; }
					if (!dup) J->cnt[lg[x].id]++;
				}
			}
	}
	return NULL;
}

int svg_events_anti_support(svg_events *t, const svg_params *p, const svg_event_params *ep_in, uint64_t n_reads, int ends,
                            const svg_mapping_result *out)
{
	const int mb = p ? p->multi_best : 0;
	svg_event_params epd;
	const svg_event_params *ep = ep_in;
	side_t *sm, *lg;
	uint32_t *cnt;
	int64_t ne, i;
	if (!t || !p || !out || ends < 1 || ends > 2 || mb < 1 || mb > 3) { svg_set_error("svg_events_anti_support: bad argument"); return SVG_E_ARG; }
	if (!ep) { svg_event_params_default(&epd); ep = &epd; }
	ne = (int64_t)t->n;
	if (ne < 1) return 0;
	/* the reads split over host threads, each with its own counters (sums: order-independent) */
	int T = svg_host_threads();
	if ((uint64_t)T > n_reads / 4096 + 1) T = (int)(n_reads / 4096 + 1);
	if (T < 1) T = 1;
	sm = malloc(sizeof(side_t) * (size_t)ne);
	lg = malloc(sizeof(side_t) * (size_t)ne);
	cnt = calloc((size_t)ne * (size_t)T, sizeof(uint32_t));
	anti_job *jobs = calloc((size_t)T, sizeof(anti_job));
	pthread_t *tid = calloc((size_t)T, sizeof(pthread_t));
	char *started = calloc((size_t)T, 1);
	if (!sm || !lg || !cnt || !jobs || !tid || !started) {
		free(sm); free(lg); free(cnt); free(jobs); free(tid); free(started);
		svg_set_error("out of memory");
		return SVG_E_NOMEM;
	}
	for (i = 0; i < ne; i++) {
		sm[i].pos = t->ev[i].small_side; sm[i].id = (uint32_t)i;
		lg[i].pos = t->ev[i].large_side; lg[i].id = (uint32_t)i;
	}
	qsort(sm, (size_t)ne, sizeof(side_t), side_cmp);
	qsort(lg, (size_t)ne, sizeof(side_t), side_cmp);
	for (int k = 0; k < T; k++) {
		anti_job *J = &jobs[k];
		J->sm = sm; J->lg = lg; J->ne = ne; J->p = p; J->ep = ep; J->out = out; J->ends = ends; J->mb = mb;
		J->r0 = n_reads * (uint64_t)k / (uint64_t)T;
		J->r1 = n_reads * (uint64_t)(k + 1) / (uint64_t)T;
		J->cnt = cnt + (size_t)ne * (size_t)k;
		/* a thread that cannot be created (thread or memory limits) scans its range inline */
		if (k) started[k] = pthread_create(&tid[k], NULL, anti_worker, J) == 0;
	}
	anti_worker(&jobs[0]);
	for (int k = 1; k < T; k++) {
		if (started[k]) pthread_join(tid[k], NULL);
		else anti_worker(&jobs[k]);
	}
	for (int k = 1; k < T; k++)
		for (i = 0; i < ne; i++) cnt[i] += cnt[(size_t)ne * (size_t)k + (size_t)i];
	for (i = 0; i < ne; i++) t->ev[i].anti_supporting_reads = (uint16_t)(t->ev[i].anti_supporting_reads + cnt[i]);
	free(sm); free(lg); free(cnt); free(jobs); free(tid); free(started);
	return 0;
}

/* events appended as given, each put in its sides' id lists (put_new_event) in order */
int svg_events_load(svg_events *t, const svg_event *ev, int64_t n)
{
	if (!t || n < 0 || (n && !ev)) { svg_set_error("svg_events_load: bad argument"); return SVG_E_ARG; }
	for (int64_t i = 0; i < n; i++) {
		const uint64_t id = new_event(t);
		t->ev[id] = ev[i];
		/* an event remove_neighbour already took out of the site lists stays out of them
		 * (core-indel.c:573-593): it keeps its slot in the array, not in a list */
		if (ev[i].event_type) put_event(t, id);
	}
	return 0;
}

int svg_events_load_sites(svg_events *t, const svg_event *ev, int64_t n, const uint32_t *pos, const uint32_t *ids,
                          const uint8_t *cap, int64_t n_sites)
{
	if (!t || n < 0 || (n && !ev) || n_sites < 0 || (n_sites && (!pos || !ids || !cap))) {
		svg_set_error("svg_events_load_sites: bad argument");
		return SVG_E_ARG;
	}
	const uint64_t base = t->n;
	for (int64_t s = 0; s < n_sites; s++)
		if (!pos[s] || cap[s] < 1 || cap[s] > EV_PER_SITE || site_find(t, pos[s])) {
			svg_set_error("svg_events_load_sites: site %lld (coordinate %u, room %u) invalid or given twice", (long long)s,
			              pos[s], (unsigned)cap[s]);
			return SVG_E_ARG;
		}
	for (int64_t i = 0; i < n; i++) {
		const uint64_t id = new_event(t);   /* (may move t->ev) */
		t->ev[id] = ev[i];
	}
	for (int64_t s = 0; s < n_sites; s++) {
		site_t *st = site_get(t, pos[s]);
		st->cap = cap[s];
		memset(st->ids, 0, sizeof st->ids);
		for (int k = 0; k < cap[s]; k++) {
			const uint32_t v = ids[s * EV_PER_SITE + k];
			if (!v) break;
			if (v > (uint64_t)n) { svg_set_error("svg_events_load_sites: site %lld lists event %u of %lld", (long long)s, v, (long long)n); return SVG_E_ARG; }
			st->ids[k] = (uint32_t)(base + v);
		}
	}
	return 0;
}

/* ------------------------------------------------------------------ remove_neighbour */
typedef struct { uint64_t *v; uint64_t n, cap; } idlist_t;

static int idlist_push(idlist_t *l, uint64_t id)
{
	if (l->n == l->cap) {
		uint64_t nc = l->cap ? 2 * l->cap : 1024;
		uint64_t *nv = realloc(l->v, nc * sizeof(uint64_t));
		if (!nv) return SVG_E_NOMEM;
		l->v = nv;
		l->cap = nc;
	}
	l->v[l->n++] = id;
	return 0;
}

/* one id out of the site list at key (remove_neighbour's second loop, core-indel.c:572-590) */
static void site_drop(svg_events *t, uint32_t key, uint64_t id)
{
	site_t *st = site_find(t, key);
	if (!st) return;
	int w = 0, k;
	for (k = 0; k < (int)st->cap && st->ids[k]; k++) {
		if (st->ids[k] - 1 == id) continue;
		st->ids[w++] = st->ids[k];
	}
	for (; w < k; w++) st->ids[w] = 0;
}

/*
 * remove_neighbour, core-indel.c:447-595 (no scRNA input, no fusion / long-deletion events): an
 * indel with an indel of the same length within 3 bases of its small side is dropped unless the
 * two are connected or it has the better quality (then the more supporting reads; on a tie the
 * one at the higher coordinate stays); a junction / fusion event without the known-event mark
 * (is_donor_found_or_annotation & 64) is dropped for a neighbour within 11 bases whose large
 * side is within 4 of the shifted one and that has more supporting reads (a tie: the neighbour
 * at the lower coordinate wins), or that has a smaller indel_at_junction over an intron of
 * about the same length.  Every decision reads the table as it was before the pass; the
 * dropped events become type 0 (CHRO_EVENT_TYPE_REMOVED) and leave their sides' id lists.
 * The arithmetic is the reference's unsigned 32-bit coordinate arithmetic.
 */
int svg_events_remove_neighbour(svg_events *t)
{
	if (!t) { svg_set_error("svg_events_remove_neighbour: NULL argument"); return SVG_E_ARG; }
	idlist_t rm = {NULL, 0, 0};
	uint64_t i, ids[EV_PER_SITE];
	int rc = 0;
	for (i = 0; i < t->n && !rc; i++) {
		const svg_event *e = &t->ev[i];
		if (e->event_type == 0) continue;
		if (e->event_type == SVG_EVENT_INDEL) {
			/* (is_ambiguous_indel_score is 0, core-indel.h:214) */
			for (int d = -3; d <= 3 && !rc; d++) {
				const int nf = search_small(t, e->small_side + (uint32_t)d, SVG_EVENT_INDEL, ids);
				for (int k = 0; k < nf && !rc; k++) {
					const svg_event *nb = &t->ev[ids[k]];
					const long long ld = (long long)nb->indel_length - e->indel_length;
					if (ld == 0 && d == 0) continue;
					if (ld != 0) continue;
					if (e->small_side - (uint32_t)(int)e->connected_previous_event_distance + 1u == nb->large_side) continue;
					if (nb->small_side - (uint32_t)(int)nb->connected_previous_event_distance + 1u == e->large_side) continue;
					if (e->large_side + (uint32_t)(int)e->connected_next_event_distance - 1u == nb->small_side) continue;
					if (nb->large_side + (uint32_t)(int)nb->connected_next_event_distance - 1u == e->small_side) continue;
					if (e->event_quality < nb->event_quality ||
					    (e->event_quality == nb->event_quality &&
					     (e->supporting_reads < nb->supporting_reads || (e->supporting_reads == nb->supporting_reads && d < 0))))
						rc = idlist_push(&rm, i);
				}
			}
		} else {
			if (e->is_donor_found_or_annotation & 64) continue;
			for (int d = -11; d <= 11 && !rc; d++) {
				if (!d) continue;
				const int nf = search_small(t, e->small_side + (uint32_t)d, SVG_EVENT_JUNCTION | SVG_EVENT_FUSION, ids);
				for (int k = 0; k < nf && !rc; k++) {
					const svg_event *nb = &t->ev[ids[k]];
					if (nb->indel_at_junction > e->indel_at_junction) continue;
					const int32_t span = (int32_t)(nb->large_side - nb->small_side + (uint32_t)(int)nb->indel_at_junction -
					                               e->large_side + e->small_side - (uint32_t)(int)e->indel_at_junction);
					if (e->indel_at_junction > nb->indel_at_junction && abs(span) <= 16)
						rc = idlist_push(&rm, i);
					else if (nb->large_side >= e->large_side - 4u + (uint32_t)d && nb->large_side <= e->large_side + 4u + (uint32_t)d &&
					         (e->supporting_reads < nb->supporting_reads || (e->supporting_reads == nb->supporting_reads && d < 0)))
						rc = idlist_push(&rm, i);
				}
			}
		}
	}
	if (rc) { free(rm.v); svg_set_error("out of memory"); return rc; }
	for (i = 0; i < rm.n; i++) {
		svg_event *e = &t->ev[rm.v[i]];
		site_drop(t, e->small_side, rm.v[i]);
		site_drop(t, e->large_side, rm.v[i]);
		e->event_type = 0;
	}
	free(rm.v);
	return 0;
}
