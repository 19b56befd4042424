/*
 * svg_sam.c -- ordered SAM emission (include/subread_sam.h).
 *
 * Replaces the ordered write of add_buffered_fragment (reference core.c:1835-1884): there every
 * iteration-two thread spins on the output lock (lock, compare last_written_fragment_number
 * with its fragment - 1, unlock, usleep(2)) until the fragments before its own are out.  Here a
 * producer never waits: its text goes into a reorder ring slot keyed by fragment number, and the
 * producer that completes the oldest unwritten fragment drains every complete fragment from
 * there on into a staging buffer that leaves in large fwrite()s.  The bytes and their order are
 * the reference's: fragments in number order, each fragment's locations in put order (one
 * thread writes all locations of its fragment, in order, core.c:2707-2782,2905-2948).
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include "svg_internal.h"
#include "subread_sam.h"

typedef struct {
	char *buf;
	size_t len, cap;
	int got;          /* locations put so far */
	int all;          /* all_locations of the fragment (0: nothing put yet) */
	int64_t span;     /* fragments the text covers (svg_sam_writer_put_block; 1 otherwise) */
} sam_slot;

/* A full staging buffer leaves the ring lock as a numbered batch: the thread that detached it
 * writes it under the file lock once every earlier batch is written (batches leave in number
 * order), so producers never wait on file I/O to put their text. */
typedef struct sam_batch {
	char *buf;
	size_t len, cap;
	uint64_t ticket;
	int flush;                /* fflush after it (the chunk's last batch) */
	struct sam_batch *next;   /* free list */
} sam_batch;

struct svg_sam_writer {
	FILE *fp;
	pthread_mutex_t mu;       /* ring, staging, tickets */
	sam_slot *ring;
	uint64_t size;          /* power of two */
	int64_t next;           /* oldest fragment not written yet */
	int64_t pending;        /* fragments with text held in the ring */
	int64_t chunk_end;      /* fragments in the chunk: flush once `next` reaches it */
	sam_batch *out;         /* staging of drained fragments */
	sam_batch *spare;       /* written batches, for reuse */
	uint64_t tickets;       /* batches detached so far */
	pthread_mutex_t wmu;      /* the FILE*; written / failed */
	pthread_cond_t wcv;
	uint64_t written;       /* batches written so far */
	int failed;
};

#define OUT_FLUSH (4u << 20)

static sam_batch *batch_new(svg_sam_writer *w)
{
	sam_batch *b = w->spare;
	if (b) { w->spare = b->next; b->len = 0; b->flush = 0; return b; }
	b = calloc(1, sizeof *b);
	if (!b) return NULL;
	b->cap = OUT_FLUSH;
	b->buf = malloc(b->cap);
	if (!b->buf) { free(b); return NULL; }
	return b;
}

/* (ring lock held) the staging buffer becomes batch `ticket`; a fresh one takes its place */
static sam_batch *out_detach(svg_sam_writer *w, int flush)
{
	sam_batch *b = w->out, *nb = batch_new(w);
	if (!nb) return NULL;
	b->ticket = w->tickets++;
	b->flush = flush;
	w->out = nb;
	return b;
}

/* (no lock held) write batch b in ticket order, then hand it back to the spares */
static int batch_write(svg_sam_writer *w, sam_batch *b)
{
	pthread_mutex_lock(&w->wmu);
	while (w->written != b->ticket) pthread_cond_wait(&w->wcv, &w->wmu);
	if (b->len && fwrite(b->buf, 1, b->len, w->fp) != b->len) w->failed = 1;
	if (b->flush && fflush(w->fp)) w->failed = 1;
	w->written++;
	const int f = w->failed;
	pthread_cond_broadcast(&w->wcv);
	pthread_mutex_unlock(&w->wmu);
	pthread_mutex_lock(&w->mu);
	b->next = w->spare;
	w->spare = b;
	pthread_mutex_unlock(&w->mu);
	return f ? SVG_E_IO : 0;
}

static int out_append(svg_sam_writer *w, const char *s, size_t n)
{
	sam_batch *o = w->out;
	if (o->len + n > o->cap) {
		size_t nc = o->cap;
		while (o->len + n > nc) nc *= 2;   /* (detached at OUT_FLUSH / 2: only a huge fragment grows it) */
		char *nb = realloc(o->buf, nc);
		if (!nb) return SVG_E_NOMEM;
		o->buf = nb;
		o->cap = nc;
	}
	memcpy(o->buf + o->len, s, n);
	o->len += n;
	return 0;
}

int svg_sam_writer_open(void *file, svg_sam_writer **out)
{
	if (!file || !out) { svg_set_error("svg_sam_writer_open: NULL argument"); return SVG_E_ARG; }
	svg_sam_writer *w = calloc(1, sizeof *w);
	if (!w) { svg_set_error("out of memory"); return SVG_E_NOMEM; }
	w->fp = (FILE *)file;
	w->size = 1024;
	w->ring = calloc(w->size, sizeof(sam_slot));
	w->chunk_end = -1;
	w->out = batch_new(w);
	if (!w->ring || !w->out) {
		if (w->out) { free(w->out->buf); free(w->out); }
		free(w->ring); free(w); svg_set_error("out of memory"); return SVG_E_NOMEM;
	}
	pthread_mutex_init(&w->mu, NULL);
	pthread_mutex_init(&w->wmu, NULL);
	pthread_cond_init(&w->wcv, NULL);
	*out = w;
	return 0;
}

/* the ring must hold fragment f: grow (re-slot by f mod size) while f - next >= size */
static int ring_reserve(svg_sam_writer *w, int64_t f)
{
	if ((uint64_t)(f - w->next) < w->size) return 0;
	uint64_t ns = w->size;
	while ((uint64_t)(f - w->next) >= ns) ns *= 2;
	sam_slot *nr = calloc(ns, sizeof(sam_slot));
	if (!nr) { svg_set_error("out of memory"); return SVG_E_NOMEM; }
	for (uint64_t i = 0; i < w->size; i++) {
		const int64_t g = w->next + (int64_t)i;     /* slots hold fragments next .. next+size-1 */
		nr[(uint64_t)g & (ns - 1)] = w->ring[(uint64_t)g & (w->size - 1)];
	}
	free(w->ring);
	w->ring = nr;
	w->size = ns;
	return 0;
}

/* move every complete fragment from `next` on to the staging buffer (ring lock held); *out gets
 * the batch to write once the lock is released (staging half full, or the chunk complete) */
static int drain(svg_sam_writer *w, sam_batch **out)
{
	int rc = 0;
	for (;;) {
		sam_slot *s = &w->ring[(uint64_t)w->next & (w->size - 1)];
		if (!s->all || s->got < s->all) break;
		if (!rc) rc = out_append(w, s->buf, s->len);
		const int64_t span = s->span > 0 ? s->span : 1;
		s->len = 0;
		s->got = s->all = 0;
		s->span = 0;
		w->next += span;
		w->pending--;
	}
	const int end = w->next == w->chunk_end;
	if (!rc && (w->out->len >= OUT_FLUSH / 2 || end) && !(*out = out_detach(w, end))) rc = SVG_E_NOMEM;
	return rc;
}

int svg_sam_writer_put(svg_sam_writer *w, int64_t fragment, int location, int all_locations, const char *text, size_t len)
{
	if (!w || fragment < 0 || all_locations < 1 || location < 0 || location >= all_locations || (len && !text)) {
		svg_set_error("svg_sam_writer_put: bad argument");
		return SVG_E_ARG;
	}
	int rc = 0;
	sam_batch *wb = NULL;
	pthread_mutex_lock(&w->mu);
	if (fragment < w->next) {
		pthread_mutex_unlock(&w->mu);
		svg_set_error("svg_sam_writer_put: fragment %lld was already written", (long long)fragment);
		return SVG_E_ARG;
	}
	if ((rc = ring_reserve(w, fragment))) { pthread_mutex_unlock(&w->mu); return rc; }
	sam_slot *s = &w->ring[(uint64_t)fragment & (w->size - 1)];
	if (!s->all) { s->all = all_locations; w->pending++; }
	if (fragment == w->next && s->got == 0 && location + 1 == all_locations) {
		/* the oldest missing fragment arriving whole: no copy through the slot */
		rc = out_append(w, text, len);
		s->got = s->all = 0;
		w->next++;
		w->pending--;
		if (!rc) rc = drain(w, &wb);
	} else {
		if (s->len + len > s->cap) {
			size_t nc = (s->len + len) * 2 + 256;
			char *nb = realloc(s->buf, nc);
			if (!nb) { pthread_mutex_unlock(&w->mu); svg_set_error("out of memory"); return SVG_E_NOMEM; }
			s->buf = nb;
			s->cap = nc;
		}
		memcpy(s->buf + s->len, text, len);
		s->len += len;
		s->got++;
		if (fragment == w->next) rc = drain(w, &wb);
	}
	pthread_mutex_unlock(&w->mu);
	if (wb) {
		const int wr = batch_write(w, wb);
		if (!rc) rc = wr;
	}
	if (rc == SVG_E_IO) svg_set_error("svg_sam_writer_put: write failed");
	else if (rc == SVG_E_NOMEM) svg_set_error("out of memory");
	return rc;
}

int svg_sam_writer_put_block(svg_sam_writer *w, int64_t first, int64_t count, const char *text, size_t len)
{
	if (!w || first < 0 || count < 1 || (len && !text)) {
		svg_set_error("svg_sam_writer_put_block: bad argument");
		return SVG_E_ARG;
	}
	int rc = 0;
	sam_batch *wb = NULL;
	pthread_mutex_lock(&w->mu);
	if (first < w->next) {
		pthread_mutex_unlock(&w->mu);
		svg_set_error("svg_sam_writer_put_block: fragment %lld was already written", (long long)first);
		return SVG_E_ARG;
	}
	if ((rc = ring_reserve(w, first))) { pthread_mutex_unlock(&w->mu); return rc; }
	sam_slot *s = &w->ring[(uint64_t)first & (w->size - 1)];
	if (s->all) {
		pthread_mutex_unlock(&w->mu);
		svg_set_error("svg_sam_writer_put_block: fragment %lld was already put", (long long)first);
		return SVG_E_ARG;
	}
	w->pending++;
	if (first == w->next) {
		/* the oldest missing fragments arriving whole: straight to the staging buffer */
		rc = out_append(w, text, len);
		w->next += count;
		w->pending--;
		if (!rc) rc = drain(w, &wb);
	} else {
		if (len > s->cap) {
			size_t nc = len * 2 + 256;
			char *nb = realloc(s->buf, nc);
			if (!nb) { w->pending--; pthread_mutex_unlock(&w->mu); svg_set_error("out of memory"); return SVG_E_NOMEM; }
			s->buf = nb;
			s->cap = nc;
		}
		memcpy(s->buf, text, len);
		s->len = len;
		s->got = s->all = 1;
		s->span = count;
	}
	pthread_mutex_unlock(&w->mu);
	if (wb) {
		const int wr = batch_write(w, wb);
		if (!rc) rc = wr;
	}
	if (rc == SVG_E_IO) svg_set_error("svg_sam_writer_put_block: write failed");
	else if (rc == SVG_E_NOMEM) svg_set_error("out of memory");
	return rc;
}

int svg_sam_writer_begin_chunk(svg_sam_writer *w, int64_t n_fragments)
{
	if (!w) return SVG_E_ARG;
	pthread_mutex_lock(&w->mu);
	const int64_t p = w->pending;
	if (!p) { w->next = 0; w->chunk_end = n_fragments; }
	pthread_mutex_unlock(&w->mu);
	if (p) { svg_set_error("svg_sam_writer_begin_chunk: %lld fragments of the last chunk incomplete", (long long)p); return SVG_E_ARG; }
	return 0;
}

int64_t svg_sam_writer_pending(svg_sam_writer *w)
{
	if (!w) return 0;
	pthread_mutex_lock(&w->mu);
	const int64_t p = w->pending;
	pthread_mutex_unlock(&w->mu);
	return p;
}

int svg_sam_writer_failed(svg_sam_writer *w)
{
	if (!w) return 0;
	pthread_mutex_lock(&w->wmu);
	const int f = w->failed;
	pthread_mutex_unlock(&w->wmu);
	return f;
}

int svg_sam_writer_close(svg_sam_writer *w)
{
	if (!w) return 0;
	/* every producer has returned: the batches they detached are written; what is staged goes now */
	pthread_mutex_lock(&w->mu);
	sam_batch *b = out_detach(w, 1);
	const int64_t p = w->pending;
	pthread_mutex_unlock(&w->mu);
	int rc = b ? batch_write(w, b) : SVG_E_NOMEM;
	for (uint64_t i = 0; i < w->size; i++) free(w->ring[i].buf);
	free(w->ring);
	for (sam_batch *q = w->spare, *nx; q; q = nx) { nx = q->next; free(q->buf); free(q); }
	if (w->out) { free(w->out->buf); free(w->out); }
	pthread_mutex_destroy(&w->mu);
	pthread_mutex_destroy(&w->wmu);
	pthread_cond_destroy(&w->wcv);
	free(w);
	if (p) { svg_set_error("svg_sam_writer_close: %lld fragments never completed", (long long)p); return SVG_E_ARG; }
	if (rc) svg_set_error("svg_sam_writer_close: write failed");
	return rc;
}

/* ---- one SAM line, byte-identical to "%s\t%d\t%s\t%u\t%d\t%s\t%s\t%u\t%d\t%s\t%s%s%s\n" */
static char *put_str(char *p, const char *s, const char *end)
{
	while (*s && p < end) *p++ = *s++;
	return *s ? NULL : p;
}

static char *put_u32(char *p, uint32_t v, const char *end)
{
	char t[10];
	int n = 0;
	do { t[n++] = (char)('0' + v % 10); v /= 10; } while (v);
	if (p + n > end) return NULL;
	while (n) *p++ = t[--n];
	return p;
}

static char *put_i32(char *p, int32_t v, const char *end)
{
	if (v < 0) {
		if (p >= end) return NULL;
		*p++ = '-';
		return put_u32(p, (uint32_t)(-(int64_t)v), end);
	}
	return put_u32(p, (uint32_t)v, end);
}

#define PUT(e) do { if (!(p = (e))) goto full; } while (0)
#define TAB() do { if (p >= end) goto full; *p++ = '\t'; } while (0)

int64_t svg_sam_format(const svg_sam_record *r, char *buf, size_t cap)
{
	if (!r || !buf) return SVG_E_ARG;
	char *p = buf;
	const char *end = buf + cap;
	PUT(put_str(p, r->qname, end)); TAB();
	PUT(put_i32(p, r->flag, end)); TAB();
	PUT(put_str(p, r->rname, end)); TAB();
	PUT(put_u32(p, r->pos, end)); TAB();
	PUT(put_i32(p, r->mapq, end)); TAB();
	PUT(put_str(p, r->cigar, end)); TAB();
	PUT(put_str(p, r->rnext, end)); TAB();
	PUT(put_u32(p, r->pnext, end)); TAB();
	PUT(put_i32(p, r->tlen, end)); TAB();
	PUT(put_str(p, r->seq, end)); TAB();
	PUT(put_str(p, r->qual, end));
	if (r->tags && r->tags[0]) {
		TAB();
		PUT(put_str(p, r->tags, end));
	}
	if (p >= end) goto full;
	*p++ = '\n';
	return (int64_t)(p - buf);
full:
	return SVG_E_ARG;
}
