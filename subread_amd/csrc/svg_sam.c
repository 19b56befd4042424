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
 *
 * BAM mode (svg_sam_writer_open_bam) is the same ordered sink over binary records
 * (svg_bam_format) that leave as BGZF blocks cut exactly where the reference's single ordered
 * stream cuts them: SamBam_writer_add_read (sambam-file.c:1704-1797) appends each record to the
 * stream's buffer and, after a committable record (the pair's second, or every single-end one)
 * that takes the buffer past 55000 bytes, SamBam_writer_add_chunk (:1193-1245) deflates it as one
 * block.  The drain cuts the same blocks; the thread that cut one deflates it with no lock held
 * (so blocks compress in parallel), then writes it in cut order.  A partial block carries over to
 * the next chunk, as the reference's buffer does, and leaves at close.
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <zlib.h>
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
	unsigned char *z;         /* BAM: the block, BGZF-compressed (zlen bytes) */
	size_t zlen;
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
	int bam;                /* BAM mode: records per location (1 single end, 2 pairs); 0 = SAM */
	int level;              /* BAM: deflate level */
};

#define OUT_FLUSH (4u << 20)
#define BAM_CUT 55000             /* sambam-file.c:1792: a block ends past 55000 bytes ... */
#define BAM_ZOUT 70000            /* ... and deflates into a 70000-byte buffer (:1213) */

/* a batch list (the blocks one drain cuts) */
typedef struct { sam_batch *head, *tail; } blist;
static void blist_push(blist *q, sam_batch *b)
{
	b->next = NULL;
	if (q->tail) q->tail->next = b;
	else q->head = b;
	q->tail = b;
}

static sam_batch *batch_new(svg_sam_writer *w)
{
	sam_batch *b = w->spare;
	if (b) { w->spare = b->next; b->len = 0; b->flush = 0; return b; }
	b = calloc(1, sizeof *b);
	if (!b) return NULL;
	b->cap = w->bam ? 2 * BAM_CUT : OUT_FLUSH;
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

/* SamBam_writer_add_chunk + SamBam_writer_chunk_header (sambam-file.c:1155-1245): the block's
 * bytes deflated raw (window bits -15, memory level 8, default strategy) into at most 70000 bytes,
 * behind the 18-byte BGZF header (mtime 0, XFL 0, OS 0xff, one BC field: block size - 1), then the
 * CRC32 and the uncompressed length */
static int bam_compress(svg_sam_writer *w, sam_batch *b)
{
	if (!b->z && !(b->z = malloc(18 + BAM_ZOUT + 8))) return SVG_E_NOMEM;
	z_stream zs;
	memset(&zs, 0, sizeof zs);
	if (deflateInit2(&zs, w->level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return SVG_E_NOMEM;
	zs.next_in = (unsigned char *)b->buf;
	zs.avail_in = (unsigned)b->len;
	zs.next_out = b->z + 18;
	zs.avail_out = BAM_ZOUT;
	deflate(&zs, Z_FINISH);
	deflateEnd(&zs);
	const unsigned csize = BAM_ZOUT - zs.avail_out;
	static const unsigned char head[16] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 66, 67, 2, 0};
	memcpy(b->z, head, 16);
	const unsigned bsize = csize + 19 + 6;
	b->z[16] = (unsigned char)bsize;
	b->z[17] = (unsigned char)(bsize >> 8);
	const uint32_t crc = (uint32_t)crc32(crc32(0, NULL, 0), (const unsigned char *)b->buf, (unsigned)b->len), isz = (uint32_t)b->len;
	memcpy(b->z + 18 + csize, &crc, 4);
	memcpy(b->z + 22 + csize, &isz, 4);
	b->zlen = 26 + (size_t)csize;
	return 0;
}

/* (no lock held) write batch b in ticket order, then hand it back to the spares */
static int batch_write(svg_sam_writer *w, sam_batch *b)
{
	int zrc = w->bam ? bam_compress(w, b) : 0;
	pthread_mutex_lock(&w->wmu);
	while (w->written != b->ticket) pthread_cond_wait(&w->wcv, &w->wmu);
	if (zrc) w->failed = 1;   /* (the ticket still moves on: later batches are not held up) */
	else if (w->bam) { if (b->zlen && fwrite(b->z, 1, b->zlen, w->fp) != b->zlen) w->failed = 1; }
	else if (b->len && fwrite(b->buf, 1, b->len, w->fp) != b->len) w->failed = 1;
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

/* (ring lock held) BAM: the text of a run of locations -- `bam` records each -- goes to the
 * open block one location at a time; a block past BAM_CUT after a location is cut (ticketed) onto q */
static int bam_append(svg_sam_writer *w, const char *s, size_t n, blist *q)
{
	size_t i = 0;
	while (i < n) {
		size_t u = 0;
		for (int k = 0; k < w->bam; k++) {
			uint32_t bs;
			if (i + u + 4 > n) return SVG_E_ARG;
			memcpy(&bs, s + i + u, 4);
			u += 4 + (size_t)bs;
		}
		if (i + u > n) return SVG_E_ARG;
		int rc = out_append(w, s + i, u);
		if (rc) return rc;
		i += u;
		if (w->out->len > BAM_CUT) {
			sam_batch *b = out_detach(w, 0);
			if (!b) return SVG_E_NOMEM;
			blist_push(q, b);
		}
	}
	return 0;
}

static int append(svg_sam_writer *w, const char *s, size_t n, blist *q)
{
	return w->bam ? bam_append(w, s, n, q) : out_append(w, s, n);
}

static int writer_new(void *file, int bam, int level, svg_sam_writer **out)
{
	if (!file || !out) { svg_set_error("svg_sam_writer_open: NULL argument"); return SVG_E_ARG; }
	svg_sam_writer *w = calloc(1, sizeof *w);
	if (!w) { svg_set_error("out of memory"); return SVG_E_NOMEM; }
	w->bam = bam;
	w->level = level;
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

int svg_sam_writer_open(void *file, svg_sam_writer **out) { return writer_new(file, 0, 0, out); }

int svg_sam_writer_open_bam(void *file, int paired, int level, svg_sam_writer **out)
{
	if (level < 0 || level > 9) { svg_set_error("svg_sam_writer_open_bam: level %d", level); return SVG_E_ARG; }
	return writer_new(file, paired ? 2 : 1, level, out);
}

int svg_sam_writer_is_bam(const svg_sam_writer *w) { return w && w->bam; }

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

/* move every complete fragment from `next` on to the staging buffer (ring lock held); q gets
 * the batches to write once the lock is released (SAM: staging half full, or the chunk complete;
 * BAM: every block cut) */
static int drain(svg_sam_writer *w, blist *q)
{
	int rc = 0;
	for (;;) {
		sam_slot *s = &w->ring[(uint64_t)w->next & (w->size - 1)];
		if (!s->all || s->got < s->all) break;
		if (!rc) rc = append(w, s->buf, s->len, q);
		const int64_t span = s->span > 0 ? s->span : 1;
		s->len = 0;
		s->got = s->all = 0;
		s->span = 0;
		w->next += span;
		w->pending--;
	}
	if (w->bam) return rc;   /* (an open block carries over to the next chunk) */
	const int end = w->next == w->chunk_end;
	if (!rc && (w->out->len >= OUT_FLUSH / 2 || end)) {
		sam_batch *b = out_detach(w, end);
		if (b) blist_push(q, b);
		else rc = SVG_E_NOMEM;
	}
	return rc;
}

/* (no lock held) the batches of q, in ticket order */
static int write_list(svg_sam_writer *w, blist *q)
{
	int rc = 0;
	for (sam_batch *b = q->head, *nx; b; b = nx) {
		nx = b->next;
		const int wr = batch_write(w, b);
		if (!rc) rc = wr;
	}
	return rc;
}

int svg_sam_writer_put(svg_sam_writer *w, int64_t fragment, int location, int all_locations, const char *text, size_t len)
{
	if (!w || fragment < 0 || all_locations < 1 || location < 0 || location >= all_locations || (len && !text)) {
		svg_set_error("svg_sam_writer_put: bad argument");
		return SVG_E_ARG;
	}
	int rc = 0;
	blist wb = {NULL, NULL};
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
		rc = append(w, text, len, &wb);
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
	const int wr = write_list(w, &wb);
	if (!rc) rc = wr;
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
	blist wb = {NULL, NULL};
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
		rc = append(w, text, len, &wb);
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
	const int wr = write_list(w, &wb);
	if (!rc) rc = wr;
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
	/* every producer has returned: the batches they detached are written; what is staged goes now
	 * (BAM: the open block, if it holds anything -- SamBam_writer_finalise_thread, sambam-file.c:2466) */
	pthread_mutex_lock(&w->mu);
	sam_batch *b = !w->bam || w->out->len ? out_detach(w, 1) : NULL;
	const int64_t p = w->pending;
	pthread_mutex_unlock(&w->mu);
	int rc = b || w->bam ? 0 : SVG_E_NOMEM;
	if (b) rc = batch_write(w, b);
	else if (w->bam && fflush(w->fp)) rc = SVG_E_IO;
	if (!rc && w->failed) rc = SVG_E_IO;
	for (uint64_t i = 0; i < w->size; i++) free(w->ring[i].buf);
	free(w->ring);
	for (sam_batch *q = w->spare, *nx; q; q = nx) { nx = q->next; free(q->buf); free(q->z); free(q); }
	if (w->out) { free(w->out->buf); free(w->out->z); free(w->out); }
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

/* ---- one BAM record, as SamBam_writer_add_read lays it out (sambam-file.c:1704-1797) */

/* SamBam_compress_cigar (sambam-file.c:1426-1458): ops of "<n><op>" up to 96 sections; the
 * covered length counts M, N and D; an unknown op character is code 8 */
static int bam_cigar(const char *cigar, uint32_t *ops, int *cover)
{
	int n = 0, v = 0, cov = 0;
	*cover = 0;
	if (cigar[0] == '*') return 0;
	for (const char *p = cigar; *p; p++) {
		const char c = *p;
		if (c >= '0' && c <= '9') { v = v * 10 + (c - '0'); continue; }
		if (c == 'M' || c == 'N' || c == 'D') cov += v;
		int op = 0;
		while (op < 8 && "MIDNSHP=X"[op] != c) op++;
		ops[n++] = ((uint32_t)v << 4) | (uint32_t)op;
		v = 0;
		if (n >= 96) break;
	}
	*cover = cov;
	return n;
}

/* SamBam_compress_additional (sambam-file.c:1478-1582): TAG:TYPE:VALUE fields separated by tabs;
 * i -> 'i' + int32 (atoi), f -> 'f' + four zero bytes (the reference converts the value into an
 * int it never stores), Z / H -> the string + NUL (cut past 780 bytes), A -> one character,
 * B -> subtype, count and the values; stops once past 750 bytes */
static int bam_tags(const char *a, char *bin)
{
	const int len = (int)strlen(a);
	int c = 0, o = 0;
	while (c < len) {
		if (c == 0 || a[c] == '\t') {
			if (a[c] == '\t') c++;
			bin[o] = a[c];
			bin[o + 1] = a[c + 1];
			const char t = a[c + 3];
			if (t == 'i' || t == 'f') {
				int dl = 0;
				while (a[dl + c + 5] != '\t' && a[dl + c + 5]) dl++;
				int32_t val = t == 'i' ? atoi(a + c + 5) : 0;
				bin[o + 2] = t;
				memcpy(bin + o + 3, &val, 4);
				o += 7;
				c += 5 + dl;
			} else if (t == 'Z' || t == 'H') {
				bin[o + 2] = t;
				o += 3;
				int sl = 0;
				c += 5;
				while (a[sl + c] != '\t' && a[sl + c]) {
					bin[o + sl] = a[sl + c];
					sl++;
					if (o + sl > 780) break;
				}
				bin[o + sl] = 0;
				o += sl + 1;
				c += sl;
			} else if (t == 'A') {
				bin[o + 2] = 'A';
				bin[o + 3] = a[c + 5];
				c += 6;
				o += 4;
			} else if (t == 'B') {
				const char ct = a[c + 5];
				const int items_at = o + 4;
				int32_t items = 0;
				bin[o + 2] = 'B';
				bin[o + 3] = ct;
				o += 8;
				c += 7;
				int last = c;
				for (;;) {
					if (a[c] == ',' || a[c] == '\t' || a[c] == 0) {
						if (c - last < 29) {
							char cell[30];
							memcpy(cell, a + last, (size_t)(c - last));
							cell[c - last] = 0;
							int32_t iv = 0;
							float fv = 0;
							if (ct == 'i') iv = atoi(cell);
							else fv = (float)atof(cell);
							if (o < 780) {
								if (ct == 'i') memcpy(bin + o, &iv, 4);
								else memcpy(bin + o, &fv, 4);
								o += 4;
								items++;
							}
						}
						last = c + 1;
					}
					if (a[c] == '\t' || a[c] == 0) break;
					c++;
				}
				memcpy(bin + items_at, &items, 4);
			} else if (c == 0) break;   /* (an unknown type in the first field: the reference spins here) */
			if (o > 750) break;
			continue;
		}
		c++;
	}
	return o;
}

/* SamBam_reg2bin (sambam-file.c:1584-1593) on the reference's int arithmetic */
static int bam_reg2bin(int beg, int end)
{
	--end;
	if (beg >> 14 == end >> 14) return ((1 << 15) - 1) / 7 + (beg >> 14);
	if (beg >> 17 == end >> 17) return ((1 << 12) - 1) / 7 + (beg >> 17);
	if (beg >> 20 == end >> 20) return ((1 << 9) - 1) / 7 + (beg >> 20);
	if (beg >> 23 == end >> 23) return ((1 << 6) - 1) / 7 + (beg >> 23);
	if (beg >> 26 == end >> 26) return ((1 << 3) - 1) / 7 + (beg >> 26);
	return 0;
}

static inline char *put_le32(char *p, uint32_t v) { memcpy(p, &v, 4); return p + 4; }

int64_t svg_bam_format(const svg_sam_record *r, int32_t refid, int32_t next_refid, int32_t read_len, char *buf, size_t cap)
{
	if (!r || !buf || read_len < 0) return SVG_E_ARG;
	uint32_t ops[96];
	int cover;
	const int nops = bam_cigar(r->cigar, ops, &cover);
	char tags[1000];
	const int tl = r->tags ? bam_tags(r->tags, tags) : 0;
	/* l_seq is the read's length: a read text holding a NUL byte encodes its bases up to the NUL only
	 * (SamBam_read2bin reads the string) -- the rest of the 4-bit field, which the reference's
	 * record leaves as whatever its stream buffer held there, is zero here */
	const int name_len = 1 + (int)strlen(r->qname), rl = read_len, tl_seq = (int)strnlen(r->seq, (size_t)read_len);
	const int32_t reclen = 32 + name_len + nops * 4 + (rl + 1) / 2 + rl + tl;
	if (cap < 4 + (size_t)reclen) return SVG_E_ARG;
	char *p = buf;
	p = put_le32(p, (uint32_t)reclen);
	const int bin = bam_reg2bin((int)(r->pos - 1u), (int)(r->pos - 1u + (uint32_t)cover));
	p = put_le32(p, (uint32_t)refid);
	p = put_le32(p, r->pos - 1u);
	p = put_le32(p, ((uint32_t)bin << 16) | ((uint32_t)r->mapq << 8) | (uint32_t)name_len);
	p = put_le32(p, ((uint32_t)r->flag << 16) | (uint32_t)nops);
	p = put_le32(p, (uint32_t)rl);
	p = put_le32(p, (uint32_t)next_refid);
	p = put_le32(p, r->pnext - 1u);
	p = put_le32(p, (uint32_t)r->tlen);
	memcpy(p, r->qname, (size_t)name_len);
	p += name_len;
	memcpy(p, ops, 4 * (size_t)nops);
	p += 4 * nops;
	/* SamBam_read2bin (:1460-1476): 4-bit codes of "=ACMGRSVTWYHKDBN", anything else 15 */
	memset(p, 0, (size_t)(rl + 1) / 2);
	for (int i = 0; i < tl_seq; i++) {
		const char c = r->seq[i];
		int code = 0;
		while (code < 15 && "=ACMGRSVTWYHKDBN"[code] != c) code++;
		if (i % 2 == 0) p[i / 2] = (char)(code << 4);
		else p[i / 2] = (char)(p[i / 2] | code);
	}
	p += (rl + 1) / 2;
	for (int i = 0; i < rl; i++) p[i] = (char)(r->qual[i] - 33);
	p += rl;
	memcpy(p, tags, (size_t)tl);
	p += tl;
	return (int64_t)(p - buf);
}
