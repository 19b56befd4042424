// svg_long.hip -- sublong's voting step on the GPU (include/subread_long.h).
//
// The reference votes one long read at a time into a 64973 x 51 table (LRMdo_one_voting_read,
// longread-mapping.c:552-560; LRMgehash_go_QQ, LRMsorted-hashtable.c:443-518): for each strand,
// each subread (every ~3 bases), each item of the subread key's equal-key run in its bucket, the
// candidate position kv = value - offset goes to row kv % 64973, where it votes for the first slot
// holding exactly kv on the same strand whose coverage end + 14 is past the offset, or else opens
// a slot if the row has fewer than 51.  That serial loop has a closed form, and the GPU computes
// the closed form for a whole batch of reads with sorts instead of replaying it:
//
//   * within one (read, strand, kv) the offsets only grow, so at most one slot of that key is
//     live at any time: the key's candidates split into SEGMENTS wherever the offset jumps by
//     >= 30 (16 + 14) over the previous one; a segment is one slot (votes = its length, coverage
//     from its first offset to its last + 16);
//   * a row only fills: a segment gets a slot iff fewer than 51 segments of its row opened
//     before it (candidate order), and its slot index is that count.
//
//   probe    thread = (read, strand, subread): offset (the reference's double stepping), the
//            16-mer key (strand 1 from the LRMreverse_read text), the equal-key run from the
//            bucket code / key-hash image for sorted buckets, go_QQ's literal search otherwise
//   expand   wave = 64 probes, lanes over the probes' runs (load-balanced): candidate c gets
//            key (read, strand, kv) and payload c
//   sort 1   radix sort by (read, strand, kv), stable: candidate order within a key
//   segment  head flags (new key or offset jump >= 30), scan, per segment (kv, strand, votes,
//            coverage) and a second key (read, row, first candidate)
//   sort 2   radix sort of the segments by (read, row, first candidate): a row's segments in
//            opening order -- a segment's rank in its row is its slot index; rank >= 51 = no slot
//   emit     the kept segments in (read, row, slot) order = LRMcopy_longvotes_to_itr's order
//   order    block = read: LRMmerge_sort by pos + coverage_start with the reference's recursion
//            (halves down to <= 6 items, selection sort there, merges taking the right run first
//            on ties; LRMhelper.c:6-43, longread-mapping.c:590-622) as rank arithmetic per level
//
// Integer work only (no MFMA): HBM-bound sorts and scattered bucket reads.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <string.h>
#include <algorithm>
#include <malloc.h>
#include <mutex>
#include <thread>
#include <vector>
#include "subread_vote.h"
#include "subread_long.h"
#include "svg_internal.h"
#include "svg_device.h"

#define LR_ROWS  64973u
#define LR_SPACE 51
#define LR_LEAF  6         // LRMmerge_sort_run: items > 6 split, else selection sort
#define LR_JOIN  30        // offset < coverage_end + 14 with coverage_end = last offset + 16

// ---------------------------------------------------------------------------------------------
// probe

struct LProbe {
	DevIndex ix;
	const char *text;
	const uint64_t *toff;     // per read of the chunk: first base in text
	const uint32_t *len;
	const uint32_t *pbase;    // n + 1: first probe of each read (2 x subreads per read)
	uint32_t n_reads;
	uint64_t n_probes;
	uint64_t *pcnt;           // run length (u64 for the scan)
	uint32_t *pfirst;         // first item of the run
	uint64_t *pmeta;          // read << 22 | strand << 21 | offset
};

// LRMreverse_read's table (LRMfile-io.c:69): A C G T U complement, every other byte 'N'
__device__ __forceinline__ char l_conv(char c)
{
	return c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : (c == 'T' || c == 'U') ? 'A' : 'N';
}
// LRMbase2int (LRMconfig.h:279)
__device__ __forceinline__ uint32_t l_b2i(char c) { return c < 'G' ? (c == 'A' ? 0u : 2u) : (c == 'G' ? 1u : 3u); }

// LRMgehash_go_QQ's search (LRMsorted-hashtable.c:455-479), literally: binary search with
// imax = items, back to the first of the equal keys, the run forward from there
__device__ __forceinline__ void l_literal(const DevIndex &x, uint32_t key, uint32_t b, uint32_t &f, uint32_t &c)
{
	f = 0;
	c = 0;
	const uint32_t base = x.bstart[b];
	const int items = (int)(x.bstart[b + 1] - base);
	if (!items) return;
	const int16_t *ck = x.keys + base;
	const int16_t k = (int16_t)(key / x.nb);
	int imin = 0, imax = items, last = 0;
	while (imin < items) {
		last = (imin + imax) / 2;
		const int16_t cur = ck[last];
		if (cur > k) imax = last - 1;
		else if (cur < k) imin = last + 1;
		else break;
		if (imax < imin) return;
	}
	while (last && ck[last - 1] == k) last--;
	int e = last;
	while (e < items && ck[e] == k) e++;
	f = base + (uint32_t)last;
	c = (uint32_t)(e - last);
}

#define LIMG_LITERAL 0
#define LIMG_CODE    1
#define LIMG_KHASH   2
template <int IMG>
__global__ void __launch_bounds__(256) long_probe_kernel(LProbe lp)
{
	const uint64_t p = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (p >= lp.n_probes) return;
	const DevIndex &x = lp.ix;
	// the probe's read: last r with pbase[r] <= p
	int lo = 0, hi = (int)lp.n_reads - 1;
	while (lo < hi) { const int m = (lo + hi + 1) >> 1; if (lp.pbase[m] <= p) lo = m; else hi = m - 1; }
	const int r = lo;
	const uint32_t local = (uint32_t)p - lp.pbase[r];
	const uint32_t S = (lp.pbase[r + 1] - lp.pbase[r]) >> 1;
	const uint32_t strand = local >= S ? 1u : 0u;
	const uint32_t i = local - strand * S;
	const int L = (int)lp.len[r];
	// LRMcalc_subread_start (longread-mapping.c:529-538) with the gap of LRMcalc_total_subreads (:526)
	int off = L - 16;
	if (i + 1 < S) {
		const double gap = (double)(uint32_t)(L - 16) * 1.0 / (double)(int)(S - 1) + 0.000001;
		off = (int)(gap * (double)(int)i);
	}
	const char *t = lp.text + lp.toff[r];
	uint32_t key = 0;
	if (strand) {
#pragma unroll
		for (int q = 0; q < 16; q++) key |= l_b2i(l_conv(t[L - 1 - off - q])) << (30 - 2 * q);
	} else {
#pragma unroll
		for (int q = 0; q < 16; q++) key |= l_b2i(t[off + q]) << (30 - 2 * q);
	}
	const uint32_t qk = key / x.nb, b = key - qk * x.nb;
	uint32_t f = 0, c = 0;
	bool literal = IMG == LIMG_LITERAL;
	if (IMG == LIMG_CODE) {
		// sorted bucket of <= 169 items: the run of key_hi = qk is [fe, ee) of the bucket
		const uint4 *c4 = x.bcode + 2 * (size_t)b;
		const uint4 u0 = c4[0], u1 = c4[1];
		const uint32_t n = u0.y & 255u;
		literal = n == 255u;
		if (!literal && n) {
			const uint64_t z[4] = {~(((uint64_t)u0.y << 32) | u0.x) & ~0xffffffffffull, ~(((uint64_t)u0.w << 32) | u0.z),
			                       ~(((uint64_t)u1.y << 32) | u1.x), ~(((uint64_t)u1.w << 32) | u1.z)};
			const int k = (int)qk;
			const int fe = k ? code_zero(z, k - 1) - 40 - (k - 1) : 0;
			const int ee = code_zero(z, k) - 40 - k;
			if (ee > fe) { f = u0.x + (uint32_t)fe; c = (uint32_t)(ee - fe); }
		}
	} else if (IMG == LIMG_KHASH) {
		literal = qk > 0xffffu || !((x.ksorted[b >> 5] >> (b & 31u)) & 1u);
		if (!literal) {
			uint2 rec;
			if (khash_find(x, key, rec)) {
				{
					const uint32_t fwd = rec.y & 0xffffu, bwd = rec.y >> 16;
					f = rec.x - bwd;
					c = fwd + bwd;
				}
			}
		}
	}
	if (literal) l_literal(x, key, b, f, c);
	lp.pcnt[p] = c;
	lp.pfirst[p] = f;
	lp.pmeta[p] = ((uint64_t)r << 22) | ((uint64_t)strand << 21) | (uint64_t)(uint32_t)off;
}

// ---------------------------------------------------------------------------------------------
// expand: wave = 64 consecutive probes, lanes stride over the probes' candidates

struct LExpand {
	const uint32_t *vals;
	const uint64_t *pcnt, *pbase_c;   // run lengths, exclusive scan (candidate base per probe)
	const uint32_t *pfirst;
	const uint64_t *pmeta;
	uint64_t n_probes;
	uint64_t *ckey;                   // read << 33 | strand << 32 | kv
	uint32_t *cval;                   // candidate index
	uint32_t *coff;                   // offset
};

__global__ void __launch_bounds__(256) long_expand_kernel(LExpand le)
{
	__shared__ uint32_t s_cb[4][64], s_first[4][64];
	__shared__ uint64_t s_meta[4][64];
	const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
	const uint64_t p0 = ((uint64_t)blockIdx.x * 4u + (uint64_t)w) * 64u;
	if (p0 >= le.n_probes) return;
	const uint64_t np = le.n_probes - p0 < 64 ? le.n_probes - p0 : 64;
	const uint64_t c0 = le.pbase_c[p0];
	const uint64_t p = p0 + (uint64_t)lane;
	if ((uint64_t)lane < np) {
		s_cb[w][lane] = (uint32_t)(le.pbase_c[p] - c0);
		s_meta[w][lane] = le.pmeta[p];
		s_first[w][lane] = le.pfirst[p];
	}
	const uint64_t total = le.pbase_c[p0 + np - 1] + le.pcnt[p0 + np - 1] - c0;
	__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
	__builtin_amdgcn_wave_barrier();
	for (uint64_t t = (uint64_t)lane; t < total; t += 64) {
		// probe j of the wave: the last j < np with s_cb[j] <= t (probes with empty runs share a
		// base with the next one, which is the one with items)
		int lo = 0, hi = (int)np - 1;
		while (lo < hi) { const int m = (lo + hi + 1) >> 1; if ((uint64_t)s_cb[w][m] <= t) lo = m; else hi = m - 1; }
		const uint64_t mj = s_meta[w][lo];
		const uint32_t off = (uint32_t)(mj & 0x1fffffu);
		const uint32_t kv = le.vals[s_first[w][lo] + (uint32_t)(t - s_cb[w][lo])] - off;
		const uint64_t c = c0 + t;
		le.ckey[c] = ((mj >> 22) << 33) | (((mj >> 21) & 1u) << 32) | (uint64_t)kv;
		le.cval[c] = (uint32_t)c;
		le.coff[c] = off;
	}
}

// ---------------------------------------------------------------------------------------------
// segments

__global__ void __launch_bounds__(256) long_head_kernel(const uint64_t *key, const uint32_t *val, const uint32_t *coff,
                                                         uint64_t n, uint32_t *head)
{
	const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (i >= n) return;
	uint32_t h = 1;
	if (i) {
		const uint64_t k = key[i], kp = key[i - 1];
		h = k != kp || coff[val[i]] >= coff[val[i - 1]] + LR_JOIN;
	}
	head[i] = h;
}

__global__ void __launch_bounds__(256) long_segstart_kernel(const uint32_t *head, const uint32_t *sid, uint64_t n,
                                                             uint32_t *sfirst)
{
	const uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (i < n && head[i]) sfirst[sid[i]] = (uint32_t)i;
}

struct LSeg {
	const uint64_t *key;
	const uint32_t *val, *coff, *sfirst;
	uint64_t n_cand, n_seg;
	uint64_t *skey;           // read << 48 | row << 32 | first candidate
	uint32_t *sidx;           // segment id
	uint4 *sdata;             // kv, coverage_start, coverage_end, votes | strand << 31
};

__global__ void __launch_bounds__(256) long_seg_kernel(LSeg ls)
{
	const uint64_t j = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (j >= ls.n_seg) return;
	const uint64_t i0 = ls.sfirst[j], i1 = j + 1 < ls.n_seg ? ls.sfirst[j + 1] : ls.n_cand;
	const uint64_t k = ls.key[i0];
	const uint32_t kv = (uint32_t)k, strand = (uint32_t)(k >> 32) & 1u;
	const uint32_t c0 = ls.val[i0];
	const uint32_t cs = ls.coff[c0], ce = ls.coff[ls.val[i1 - 1]] + 16u;
	const uint32_t votes = (uint32_t)(i1 - i0);
	ls.skey[j] = ((k >> 33) << 48) | ((uint64_t)(kv % LR_ROWS) << 32) | (uint64_t)c0;
	ls.sidx[j] = (uint32_t)j;
	ls.sdata[j] = make_uint4(kv, cs, ce, (votes & 0x7fffffffu) | (strand << 31));
}

// rank of sorted segment t in its (read, row) group; kept iff < 51
__device__ __forceinline__ int l_rank(const uint64_t *skey, uint64_t t)
{
	const uint64_t g = skey[t] >> 32;
	uint64_t lo = t >= LR_SPACE ? t - LR_SPACE : 0, hi = t;   // first index of the group within [lo, t]
	while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if ((skey[m] >> 32) == g) hi = m; else lo = m + 1; }
	return (int)(t - lo);
}

__global__ void __launch_bounds__(256) long_keep_kernel(const uint64_t *skey, uint64_t n, uint32_t *keep)
{
	const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (t >= n) return;
	keep[t] = l_rank(skey, t) < LR_SPACE;
}

struct LEmit {
	const uint64_t *skey;
	const uint32_t *sidx, *keep, *kpos;
	const uint4 *sdata;
	uint64_t n_seg;
	svg_long_vote *out;
};

__global__ void __launch_bounds__(256) long_emit_kernel(LEmit le)
{
	const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
	if (t >= le.n_seg || !le.keep[t]) return;
	const uint64_t k = le.skey[t];
	const uint4 d = le.sdata[le.sidx[t]];
	svg_long_vote v;
	v.pos = d.x;
	v.coverage_start = d.y;
	v.coverage_end = d.z;
	v.votes = (uint16_t)(d.w & 0xffffu);
	v.negative = (uint8_t)(d.w >> 31);
	v._pad = 0;
	v.slot = (uint32_t)(((k >> 32) & 0xffffu) << 16) | (uint32_t)l_rank(le.skey, t);
	le.out[le.kpos[t]] = v;
}

// ---------------------------------------------------------------------------------------------
// order: LRMmerge_sort by sorting_vote_locations = pos + coverage_start, block = read

// the node of depth d containing item k of an n-item sort (false: k's leaf is shallower)
__device__ __forceinline__ bool l_node(uint32_t n, uint32_t k, int d, uint32_t &start, uint32_t &items)
{
	start = 0;
	items = n;
	for (int q = 0; q < d; q++) {
		if (items <= LR_LEAF) return false;
		const uint32_t half = items >> 1;
		if (k < start + half) items = half;
		else { start += half; items -= half; }
	}
	return true;
}

__global__ void __launch_bounds__(256) long_order_kernel(const svg_long_vote *votes, const uint64_t *vstart, uint32_t *akey,
                                                          uint32_t *aidx, uint32_t *bkey, uint32_t *bidx, uint32_t *order)
{
	const uint64_t base = vstart[blockIdx.x];
	const uint32_t n = (uint32_t)(vstart[blockIdx.x + 1] - base);
	if (n == 0) return;
	uint32_t *AK = akey + base, *AI = aidx + base, *BK = bkey + base, *BI = bidx + base;
	for (uint32_t k = threadIdx.x; k < n; k += 256) {
		const svg_long_vote v = votes[base + k];
		AK[k] = v.pos + v.coverage_start;
		AI[k] = k;
	}
	__syncthreads();
	// depth of the deepest split (the larger half is always the right one)
	int D = 0;
	for (uint32_t it = n; it > LR_LEAF; it -= it >> 1) D++;
	// leaves: LRMbasic_sort_run (LRMhelper.c:6-19) -- selection sort with exchanges
	for (uint32_t k = threadIdx.x; k < n; k += 256) {
		uint32_t s = 0, m = n;
		while (m > LR_LEAF) { const uint32_t h = m >> 1; if (k < s + h) m = h; else { s += h; m -= h; } }
		if (k != s) continue;
		for (uint32_t i = s; i + 1 < s + m; i++) {
			uint32_t mj = i;
			for (uint32_t j = i + 1; j < s + m; j++)
				if (AK[mj] > AK[j]) mj = j;
			if (mj != i) {
				const uint32_t tk = AK[i], ti = AI[i];
				AK[i] = AK[mj]; AI[i] = AI[mj];
				AK[mj] = tk; AI[mj] = ti;
			}
		}
	}
	__syncthreads();
	// merges, deepest level first (LRM_longvote_location_merge: the left run's item goes first
	// only when it is strictly smaller)
	for (int d = D - 1; d >= 0; d--) {
		for (uint32_t k = threadIdx.x; k < n; k += 256) {
			uint32_t s, m;
			const uint32_t key = AK[k], idx = AI[k];
			uint32_t pos = k;
			if (l_node(n, k, d, s, m) && m > LR_LEAF) {
				const uint32_t h = m >> 1;
				if (k < s + h) {
					// right items <= key go before it
					uint32_t lo = s + h, hi = s + m;
					while (lo < hi) { const uint32_t q = (lo + hi) >> 1; if (AK[q] <= key) lo = q + 1; else hi = q; }
					pos = k + (lo - (s + h));
				} else {
					// left items < key go before it
					uint32_t lo = s, hi = s + h;
					while (lo < hi) { const uint32_t q = (lo + hi) >> 1; if (AK[q] < key) lo = q + 1; else hi = q; }
					pos = s + (k - (s + h)) + (lo - s);
				}
			}
			BK[pos] = key;
			BI[pos] = idx;
		}
		__syncthreads();
		uint32_t *t;
		t = AK; AK = BK; BK = t;
		t = AI; AI = BI; BI = t;
	}
	for (uint32_t k = threadIdx.x; k < n; k += 256) order[base + k] = AI[k];
}

// read r's slots start at vstart[r]: the first segment of read r in the sorted order, counted in
// kept segments before it
__global__ void __launch_bounds__(256) long_vstart_kernel(const uint64_t *skey, const uint32_t *kpos, uint64_t G, uint64_t K,
                                                           uint32_t n, uint64_t *vstart)
{
	const uint32_t r = blockIdx.x * 256u + threadIdx.x;
	if (r > n) return;
	const uint64_t key = (uint64_t)r << 48;
	uint64_t lo = 0, hi = G;
	while (lo < hi) { const uint64_t m = (lo + hi) >> 1; if (skey[m] < key) lo = m + 1; else hi = m; }
	vstart[r] = lo < G ? (uint64_t)kpos[lo] : K;
}

// ---------------------------------------------------------------------------------------------
// host

// grow-only device arenas and pinned staging of the handle (svg_index::lws)
struct svg_longws {
	void *dA; size_t capA;     // probe phase: text, read table, probe arrays, scan temp
	void *dB; size_t capB;     // candidate phase: keys / payloads / segments, sort and scan temps
	void *hs[2]; size_t hcap;  // pinned staging of the uploads (in pieces)
	hipEvent_t ev[2];
	// the chunk's results by chunk parity: device slots / orders / read starts, their pinned copy,
	// the download stream and its events -- chunk c's download and host copy run while chunk c+1
	// is on the device
	void *dO[2]; size_t capO[2];
	void *hO[2]; size_t hcapO[2];
	hipStream_t down;
	hipEvent_t ev_res[2], ev_down[2];
};

namespace { void long_cache_release(); }

void svg_long_ws_free(svg_index *h)
{
	// the result-page cache (below) goes with the handle that filled it: a process that closes its
	// index does not keep GBs of freed long-read results
	long_cache_release();
	svg_longws *w = h->lws;
	if (!w) return;
	if (w->down) hipStreamSynchronize(w->down);
	hipFree(w->dA); hipFree(w->dB);
	for (int i = 0; i < 2; i++) {
		if (w->hs[i]) hipHostFree(w->hs[i]);
		if (w->ev[i]) hipEventDestroy(w->ev[i]);
		hipFree(w->dO[i]);
		if (w->hO[i]) hipHostFree(w->hO[i]);
		if (w->ev_res[i]) hipEventDestroy(w->ev_res[i]);
		if (w->ev_down[i]) hipEventDestroy(w->ev_down[i]);
		h->device_bytes -= w->capO[i];
	}
	if (w->down) hipStreamDestroy(w->down);
	h->device_bytes -= w->capA + w->capB;
	free(w);
	h->lws = NULL;
}

namespace {
// bump allocation inside an arena (a dry run with base NULL measures it)
struct Carve {
	char *base;
	size_t off;
	template <class T> T *take(size_t n)
	{
		off = (off + 255) & ~(size_t)255;
		T *p = (T *)(base ? base + off : NULL);
		off += n * sizeof(T) + 64;
		return p;
	}
};

int arena(svg_index *h, void **p, size_t *cap, size_t need)
{
	if (need <= *cap) return 0;
	if (*p) { HIPCHK(hipStreamSynchronize(h->stream)); hipFree(*p); h->device_bytes -= *cap; }
	*p = NULL;
	*cap = 0;
	need += need / 4;
	if (dmalloc(h, p, need)) return SVG_E_NOMEM;
	*cap = need;
	return 0;
}

inline uint32_t lr_subreads(uint32_t L)   // LRMcalc_total_subreads, longread-mapping.c:516-524
{
	if (L < 16) return 0;
	const uint32_t m = (L - 16 + 1) / 3;
	return m < 1200000u ? m : 1200000u;
}

inline unsigned blocks_of(uint64_t n, unsigned per) { return (unsigned)((n + per - 1) / per); }

#define LCHK(x) do { if ((x) != hipSuccess) { svg_set_error("svg_long_vote_batch: HIP error %s at %s:%d", hipGetErrorString(hipGetLastError()), __FILE__, __LINE__); return SVG_E_DEVICE; } } while (0)

const size_t PIECE = 64ull << 20;   // bytes per staged transfer

// memcpy split over the host pool's thread count
void par_copy(void *dst, const void *src, size_t n, int T)
{
	if (n < (4u << 20) || T < 2) { memcpy(dst, src, n); return; }
	std::vector<std::thread> th;
	const size_t part = (n / (size_t)T + 4095) & ~(size_t)4095;
	for (int t = 0; t < T; t++) {
		const size_t a = (size_t)t * part;
		if (a >= n) break;
		const size_t b = a + part < n ? a + part : n;
		th.emplace_back([=] { memcpy((char *)dst + a, (const char *)src + a, b - a); });
	}
	for (auto &x : th) x.join();
}

// One freed result's arrays are kept for the next call (process-wide): a batch's slots are
// ~24 B each (GBs for long-read batches), and handing the same pages back avoids unmapping them
// in svg_long_free and faulting fresh ones in during the next download.
std::mutex g_cache_mu;
void *g_cache_v = NULL, *g_cache_o = NULL;

void long_cache_release()
{
	std::lock_guard<std::mutex> lk(g_cache_mu);
	free(g_cache_v);
	free(g_cache_o);
	g_cache_v = g_cache_o = NULL;
}

struct LOut {
	svg_long_vote *votes;
	uint32_t *order;
	uint64_t n, cap;
	void adopt_cache()
	{
		std::lock_guard<std::mutex> lk(g_cache_mu);
		if (!g_cache_v || !g_cache_o) return;
		votes = (svg_long_vote *)g_cache_v;
		order = (uint32_t *)g_cache_o;
		const uint64_t cv = malloc_usable_size(votes) / sizeof(svg_long_vote), co = malloc_usable_size(order) / 4;
		cap = cv < co ? cv : co;
		g_cache_v = g_cache_o = NULL;
	}
	int reserve(uint64_t add)
	{
		if (n + add <= cap) return 0;
		const uint64_t nc = (n + add) + (n + add) / 2 + 4096;
		svg_long_vote *v = (svg_long_vote *)realloc(votes, sizeof(svg_long_vote) * nc);
		if (v) votes = v;
		uint32_t *o = (uint32_t *)realloc(order, 4 * nc);
		if (o) order = o;
		if (!v || !o) { svg_set_error("svg_long_vote_batch: out of host memory"); return SVG_E_NOMEM; }
		cap = nc;
		return 0;
	}
};

// one chunk of reads [r0, r1): appends its slots, orders and per-read counts
// the host side of a chunk's download: wait for its pinned copy, then copy it into the result
struct Pending {
	std::thread th;
	bool active = false;
	void join() { if (active) { th.join(); active = false; } }
};

int long_chunk(svg_index *h, const svg_long_reads *R, uint64_t r0, uint64_t r1, const uint64_t cand_cap, LOut &res,
               std::vector<uint64_t> &counts, bool *too_big, int T, int par, Pending &prev)
{
	hipStream_t st = h->stream;
	svg_longws *w = h->lws;
	const uint32_t n = (uint32_t)(r1 - r0);
	*too_big = false;
	const bool dbg = (svg_get_option("debug") & 4) != 0;
	auto now = [] { struct timespec ts; clock_gettime(CLOCK_MONOTONIC, &ts); return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6; };
	const double t0 = dbg ? now() : 0;
	double t_up = 0, t_probe = 0, t_seg = 0, t_keep = 0, t_dev = 0;
	std::vector<uint64_t> toff(n + 1);
	std::vector<uint32_t> len(n), pbase(n + 1);
	uint64_t tb = 0, P = 0;
	for (uint32_t i = 0; i < n; i++) {
		const uint32_t L = R->lens[r0 + i];
		toff[i] = tb;
		len[i] = L;
		tb += L;
		pbase[i] = (uint32_t)P;
		P += 2ull * lr_subreads(L);
	}
	toff[n] = tb;
	pbase[n] = (uint32_t)P;
	if (P == 0) { for (uint32_t i = 0; i < n; i++) counts[r0 + i] = 0; return 0; }
	// ---- probe phase
	size_t scan1 = 0;
	LCHK(hipcub::DeviceScan::ExclusiveSum(NULL, scan1, (uint64_t *)NULL, (uint64_t *)NULL, (int)P, st));
	Carve ca = {NULL, 0};
	for (int pass = 0; pass < 2; pass++) {
		if (pass) { if (int e = arena(h, &w->dA, &w->capA, ca.off)) return e; ca.base = (char *)w->dA; ca.off = 0; }
		ca.take<char>(tb + 16); ca.take<uint64_t>(n); ca.take<uint32_t>(n); ca.take<uint32_t>(n + 1);
		ca.take<uint64_t>(P); ca.take<uint64_t>(P); ca.take<uint64_t>(P); ca.take<uint32_t>(P); ca.take<char>(scan1);
	}
	ca.off = 0;
	char *d_text = ca.take<char>(tb + 16);
	uint64_t *d_toff = ca.take<uint64_t>(n);
	uint32_t *d_len = ca.take<uint32_t>(n), *d_pbase = ca.take<uint32_t>(n + 1);
	uint64_t *d_pcnt = ca.take<uint64_t>(P), *d_pcb = ca.take<uint64_t>(P), *d_pmeta = ca.take<uint64_t>(P);
	uint32_t *d_pfirst = ca.take<uint32_t>(P);
	void *d_tmp1 = ca.take<char>(scan1);
	// the chunk's text, read after read, through the pinned staging
	for (uint64_t a = 0; a < tb; a += PIECE) {
		const uint64_t b = a + PIECE < tb ? a + PIECE : tb;
		const int k = (int)((a / PIECE) & 1);
		LCHK(hipEventSynchronize(w->ev[k]));   // the buffer's previous transfer is done
		char *stg = (char *)w->hs[k];
		uint32_t i = (uint32_t)(std::upper_bound(toff.begin(), toff.end(), a) - toff.begin()) - 1;
		for (uint64_t o = a; o < b; i++) {
			const uint64_t e = toff[i + 1] < b ? toff[i + 1] : b;
			par_copy(stg + (o - a), R->seq + R->offsets[r0 + i] + (o - toff[i]), e - o, e - o >= (16u << 20) ? T : 1);
			o = e;
		}
		LCHK(hipMemcpyAsync(d_text + a, stg, b - a, hipMemcpyHostToDevice, st));
		LCHK(hipEventRecord(w->ev[k], st));
	}
	LCHK(hipMemcpyAsync(d_toff, toff.data(), 8ull * n, hipMemcpyHostToDevice, st));
	LCHK(hipMemcpyAsync(d_len, len.data(), 4ull * n, hipMemcpyHostToDevice, st));
	LCHK(hipMemcpyAsync(d_pbase, pbase.data(), 4ull * (n + 1), hipMemcpyHostToDevice, st));
	if (dbg) { LCHK(hipStreamSynchronize(st)); t_up = now(); }
	LProbe lp;
	lp.ix = h->dix; lp.text = d_text; lp.toff = d_toff; lp.len = d_len; lp.pbase = d_pbase; lp.n_reads = n;
	lp.n_probes = P; lp.pcnt = d_pcnt; lp.pfirst = d_pfirst; lp.pmeta = d_pmeta;
	const bool lit = svg_get_option("keys_literal") != 0;
	if (!lit && h->dix.bcode) hipLaunchKernelGGL(long_probe_kernel<LIMG_CODE>, dim3(blocks_of(P, 256)), dim3(256), 0, st, lp);
	else if (!lit && h->dix.khash && h->dix.ksorted)
		hipLaunchKernelGGL(long_probe_kernel<LIMG_KHASH>, dim3(blocks_of(P, 256)), dim3(256), 0, st, lp);
	else hipLaunchKernelGGL(long_probe_kernel<LIMG_LITERAL>, dim3(blocks_of(P, 256)), dim3(256), 0, st, lp);
	LCHK(hipGetLastError());
	LCHK(hipcub::DeviceScan::ExclusiveSum(d_tmp1, scan1, d_pcnt, d_pcb, (int)P, st));
	uint64_t last[2];
	LCHK(hipMemcpyAsync(&last[0], d_pcb + P - 1, 8, hipMemcpyDeviceToHost, st));
	LCHK(hipMemcpyAsync(&last[1], d_pcnt + P - 1, 8, hipMemcpyDeviceToHost, st));
	LCHK(hipStreamSynchronize(st));
	const uint64_t C = last[0] + last[1];
	if (dbg) t_probe = now();
	if (C > cand_cap && n > 1) { *too_big = true; return 0; }
	if (C >= 0x7fffffffull) { svg_set_error("svg_long_vote_batch: read %llu has %llu candidates", (unsigned long long)r0, (unsigned long long)C); return SVG_E_UNSUPPORTED; }
	if (C == 0) { for (uint32_t i = 0; i < n; i++) counts[r0 + i] = 0; return 0; }
	// ---- candidate phase (segments and slots are bounded by the candidates)
	int rbits = 1;
	while ((1u << rbits) < n) rbits++;
	size_t t_sort1 = 0, t_scan = 0, t_sort2 = 0;
	LCHK(hipcub::DeviceRadixSort::SortPairs(NULL, t_sort1, (uint64_t *)NULL, (uint64_t *)NULL, (uint32_t *)NULL, (uint32_t *)NULL,
	                                        (int)C, 0, 33 + rbits, st));
	LCHK(hipcub::DeviceScan::ExclusiveSum(NULL, t_scan, (uint32_t *)NULL, (uint32_t *)NULL, (int)C, st));
	LCHK(hipcub::DeviceRadixSort::SortPairs(NULL, t_sort2, (uint64_t *)NULL, (uint64_t *)NULL, (uint32_t *)NULL, (uint32_t *)NULL,
	                                        (int)C, 0, 48 + rbits, st));
	size_t t_max = t_sort1 > t_scan ? t_sort1 : t_scan;
	t_max = t_max > t_sort2 ? t_max : t_sort2;
	Carve cb = {NULL, 0};
	uint64_t *d_ck = NULL, *d_ck2 = NULL, *d_sk = NULL, *d_sk2 = NULL, *d_vs = NULL;
	uint32_t *d_cv = NULL, *d_cv2 = NULL, *d_coff = NULL, *d_head = NULL, *d_sid = NULL, *d_si = NULL, *d_si2 = NULL, *d_ord = NULL;
	uint4 *d_sd = NULL;
	svg_long_vote *d_out = NULL;
	void *d_tmp = NULL;
	for (int pass = 0; pass < 2; pass++) {
		if (pass) { if (int e = arena(h, &w->dB, &w->capB, cb.off)) return e; cb.base = (char *)w->dB; cb.off = 0; }
		d_ck = cb.take<uint64_t>(C); d_ck2 = cb.take<uint64_t>(C); d_cv = cb.take<uint32_t>(C); d_cv2 = cb.take<uint32_t>(C);
		d_coff = cb.take<uint32_t>(C); d_head = cb.take<uint32_t>(C); d_sid = cb.take<uint32_t>(C);
		d_sk = cb.take<uint64_t>(C); d_sk2 = cb.take<uint64_t>(C); d_si = cb.take<uint32_t>(C); d_si2 = cb.take<uint32_t>(C);
		d_sd = cb.take<uint4>(C);
		d_tmp = cb.take<char>(t_max);
	}
	LExpand le;
	le.vals = h->dix.vals; le.pcnt = d_pcnt; le.pbase_c = d_pcb; le.pfirst = d_pfirst; le.pmeta = d_pmeta; le.n_probes = P;
	le.ckey = d_ck; le.cval = d_cv; le.coff = d_coff;
	hipLaunchKernelGGL(long_expand_kernel, dim3(blocks_of(P, 256)), dim3(256), 0, st, le);
	LCHK(hipGetLastError());
	// sort 1: (read, strand, kv), stable
	size_t tb1 = t_max;
	LCHK(hipcub::DeviceRadixSort::SortPairs(d_tmp, tb1, d_ck, d_ck2, d_cv, d_cv2, (int)C, 0, 33 + rbits, st));
	hipLaunchKernelGGL(long_head_kernel, dim3(blocks_of(C, 256)), dim3(256), 0, st, d_ck2, d_cv2, d_coff, C, d_head);
	LCHK(hipGetLastError());
	size_t tb2 = t_max;
	LCHK(hipcub::DeviceScan::ExclusiveSum(d_tmp, tb2, d_head, d_sid, (int)C, st));
	uint32_t lh[2];
	LCHK(hipMemcpyAsync(&lh[0], d_sid + C - 1, 4, hipMemcpyDeviceToHost, st));
	LCHK(hipMemcpyAsync(&lh[1], d_head + C - 1, 4, hipMemcpyDeviceToHost, st));
	LCHK(hipStreamSynchronize(st));
	const uint64_t G = (uint64_t)lh[0] + lh[1];
	if (dbg) t_seg = now();
	uint32_t *d_sfirst = d_cv;   // the first sort's input payloads are free now
	hipLaunchKernelGGL(long_segstart_kernel, dim3(blocks_of(C, 256)), dim3(256), 0, st, d_head, d_sid, C, d_sfirst);
	LCHK(hipGetLastError());
	LSeg ls;
	ls.key = d_ck2; ls.val = d_cv2; ls.coff = d_coff; ls.sfirst = d_sfirst; ls.n_cand = C; ls.n_seg = G;
	ls.skey = d_sk; ls.sidx = d_si; ls.sdata = d_sd;
	hipLaunchKernelGGL(long_seg_kernel, dim3(blocks_of(G, 256)), dim3(256), 0, st, ls);
	LCHK(hipGetLastError());
	// sort 2: (read, row, first candidate)
	size_t tb3 = t_max;
	LCHK(hipcub::DeviceRadixSort::SortPairs(d_tmp, tb3, d_sk, d_sk2, d_si, d_si2, (int)G, 0, 48 + rbits, st));
	uint32_t *d_keep = d_head, *d_kpos = d_sid;   // G <= C
	hipLaunchKernelGGL(long_keep_kernel, dim3(blocks_of(G, 256)), dim3(256), 0, st, d_sk2, G, d_keep);
	LCHK(hipGetLastError());
	size_t tb4 = t_max;
	LCHK(hipcub::DeviceScan::ExclusiveSum(d_tmp, tb4, d_keep, d_kpos, (int)G, st));
	uint32_t lk[2];
	LCHK(hipMemcpyAsync(&lk[0], d_kpos + G - 1, 4, hipMemcpyDeviceToHost, st));
	LCHK(hipMemcpyAsync(&lk[1], d_keep + G - 1, 4, hipMemcpyDeviceToHost, st));
	LCHK(hipStreamSynchronize(st));
	const uint64_t K = (uint64_t)lk[0] + lk[1];
	if (dbg) t_keep = now();
	// this chunk's results go to the parity's output buffers (the previous chunk's may still be on
	// their way to the host)
	Carve co = {NULL, 0};
	for (int pass = 0; pass < 2; pass++) {
		if (pass) { if (int e = arena(h, &w->dO[par], &w->capO[par], co.off)) return e; co.base = (char *)w->dO[par]; co.off = 0; }
		d_vs = co.take<uint64_t>(n + 1); d_out = co.take<svg_long_vote>(K); d_ord = co.take<uint32_t>(K);
	}
	LEmit em;
	em.skey = d_sk2; em.sidx = d_si2; em.keep = d_keep; em.kpos = d_kpos; em.sdata = d_sd; em.n_seg = G; em.out = d_out;
	hipLaunchKernelGGL(long_emit_kernel, dim3(blocks_of(G, 256)), dim3(256), 0, st, em);
	LCHK(hipGetLastError());
	hipLaunchKernelGGL(long_vstart_kernel, dim3(blocks_of(n + 1, 256)), dim3(256), 0, st, d_sk2, d_kpos, G, K, n, d_vs);
	LCHK(hipGetLastError());
	// the order kernel's ping-pong arrays reuse the candidate buffers (K <= C)
	hipLaunchKernelGGL(long_order_kernel, dim3(n), dim3(256), 0, st, d_out, d_vs, (uint32_t *)d_ck, d_coff,
	                   (uint32_t *)d_ck2, d_cv2, d_ord);
	LCHK(hipGetLastError());
	LCHK(hipEventRecord(w->ev_res[par], st));
	if (dbg) { LCHK(hipStreamSynchronize(st)); t_dev = now(); }
	// the previous chunk's host copy is done before the result grows (realloc) or its staging is reused
	prev.join();
	if (int e = res.reserve(K)) return e;
	const size_t bytes = 8ull * (n + 1) + (sizeof(svg_long_vote) + 4) * K;
	if (w->hcapO[par] < bytes) {
		if (w->hO[par]) hipHostFree(w->hO[par]);
		w->hO[par] = NULL;
		w->hcapO[par] = 0;
		const size_t cap = bytes + bytes / 4;
		if (hipHostMalloc(&w->hO[par], cap, hipHostMallocDefault) != hipSuccess) { svg_set_error("svg_long_vote_batch: pinned staging of %zu bytes", cap); return SVG_E_NOMEM; }
		w->hcapO[par] = cap;
	}
	char *hv = (char *)w->hO[par];
	LCHK(hipStreamWaitEvent(w->down, w->ev_res[par], 0));
	LCHK(hipMemcpyAsync(hv, d_vs, 8ull * (n + 1), hipMemcpyDeviceToHost, w->down));
	LCHK(hipMemcpyAsync(hv + 8ull * (n + 1), d_out, sizeof(svg_long_vote) * K, hipMemcpyDeviceToHost, w->down));
	LCHK(hipMemcpyAsync(hv + 8ull * (n + 1) + sizeof(svg_long_vote) * K, d_ord, 4ull * K, hipMemcpyDeviceToHost, w->down));
	LCHK(hipEventRecord(w->ev_down[par], w->down));
	svg_long_vote *dst_v = res.votes + res.n;
	uint32_t *dst_o = res.order + res.n;
	res.n += K;
	hipEvent_t ev = w->ev_down[par];
	uint64_t *cnt = counts.data() + r0;
	const double t_issue = dbg ? now() : 0;
	prev.th = std::thread([=] {
		hipEventSynchronize(ev);
		const uint64_t *vs = (const uint64_t *)hv;
		for (uint32_t i = 0; i < n; i++) cnt[i] = vs[i + 1] - vs[i];
		par_copy(dst_v, hv + 8ull * (n + 1), sizeof(svg_long_vote) * K, T);
		par_copy(dst_o, hv + 8ull * (n + 1) + sizeof(svg_long_vote) * K, 4ull * K, T);
	});
	prev.active = true;
	if (dbg)
		fprintf(stderr, "[svg_long] reads %u probes %llu candidates %llu segments %llu slots %llu | ms: upload %.1f probe %.1f "
		        "sort1+segments %.1f sort2+keep %.1f emit+order %.1f prev-copy-wait+issue %.1f\n", n, (unsigned long long)P,
		        (unsigned long long)C, (unsigned long long)G, (unsigned long long)K, t_up - t0, t_probe - t_up, t_seg - t_probe,
		        t_keep - t_seg, t_dev - t_keep, t_issue - t_dev);
	return 0;
}
}  // namespace

extern "C" void svg_long_free(svg_long_result *r)
{
	if (!r) return;
	free(r->vstart);
	{
		// keep the larger arrays for the next call, free the others
		std::lock_guard<std::mutex> lk(g_cache_mu);
		void *v = r->votes, *o = r->order;
		if (v && o && (!g_cache_v || malloc_usable_size(v) > malloc_usable_size(g_cache_v))) {
			std::swap(v, g_cache_v);
			std::swap(o, g_cache_o);
		}
		free(v);
		free(o);
	}
	memset(r, 0, sizeof *r);
}

extern "C" int svg_long_vote_batch(svg_index *h, const svg_long_reads *R, svg_long_result *out)
{
	if (!h || !R || !out) { svg_set_error("svg_long_vote_batch: NULL argument"); return SVG_E_ARG; }
	memset(out, 0, sizeof *out);
	if (R->n_reads && (!R->seq || !R->offsets || !R->lens)) { svg_set_error("svg_long_vote_batch: NULL read buffer"); return SVG_E_ARG; }
	for (uint64_t r = 0; r < R->n_reads; r++)
		if (R->lens[r] > SVG_LONG_READ_KEEP) {
			svg_set_error("svg_long_vote_batch: read %llu has %u bases (the reference keeps at most %d)",
			              (unsigned long long)r, R->lens[r], SVG_LONG_READ_KEEP);
			return SVG_E_ARG;
		}
	HIPCHK(hipSetDevice(h->device));
	if (h->last_pending) HIPCHK(hipStreamWaitEvent(h->stream, h->ev_last, 0));
	if (!h->lws) {
		svg_longws *w = (svg_longws *)calloc(1, sizeof(svg_longws));
		if (!w) { svg_set_error("out of host memory"); return SVG_E_NOMEM; }
		h->lws = w;
		for (int i = 0; i < 2; i++) {
			HIPCHK(hipHostMalloc(&w->hs[i], PIECE, hipHostMallocDefault));
			HIPCHK(hipEventCreateWithFlags(&w->ev[i], hipEventDisableTiming));
		}
		w->hcap = PIECE;
		HIPCHK(hipStreamCreateWithFlags(&w->down, hipStreamNonBlocking));
		for (int i = 0; i < 2; i++) {
			HIPCHK(hipEventCreateWithFlags(&w->ev_res[i], hipEventDisableTiming));
			HIPCHK(hipEventCreateWithFlags(&w->ev_down[i], hipEventDisableTiming));
		}
	}
	const int T = svg_host_threads();
	// chunks: <= 65535 reads (16-bit read field of the segment key), <= 32M probes
	const uint64_t pcap = svg_get_option("long_probes") > 0 ? (uint64_t)svg_get_option("long_probes") : (32ull << 20);
	const uint64_t ccap = 256ull << 20;
	LOut res = {NULL, NULL, 0, 0};
	res.adopt_cache();
	std::vector<uint64_t> counts(R->n_reads + 1, 0);
	Pending pend;
	int par = 0;
	uint64_t r0 = 0;
	while (r0 < R->n_reads) {
		uint64_t r1 = r0, P = 0;
		while (r1 < R->n_reads && r1 - r0 < 65535) {
			const uint64_t p = 2ull * lr_subreads(R->lens[r1]);
			if (r1 > r0 && P + p > pcap) break;
			P += p;
			r1++;
		}
		for (;;) {
			bool big = false;
			const int rc = long_chunk(h, R, r0, r1, ccap, res, counts, &big, T, par, pend);
			if (rc) { pend.join(); free(res.votes); free(res.order); return rc; }
			if (!big) break;
			if (svg_get_option("debug") & 4) fprintf(stderr, "[svg_long] split %llu reads\n", (unsigned long long)(r1 - r0));
			r1 = r0 + (r1 - r0) / 2;   // too many candidates: half the reads
		}
		r0 = r1;
		par ^= 1;
	}
	pend.join();
	if (res.reserve(1)) { free(res.votes); free(res.order); return SVG_E_NOMEM; }
	out->n_reads = R->n_reads;
	out->votes = res.votes;
	out->order = res.order;
	out->vstart = (uint64_t *)malloc(8 * (R->n_reads + 1));
	if (!out->vstart) { svg_long_free(out); svg_set_error("out of host memory"); return SVG_E_NOMEM; }
	out->vstart[0] = 0;
	for (uint64_t r = 0; r < R->n_reads; r++) out->vstart[r + 1] = out->vstart[r] + counts[r];
	return 0;
}
