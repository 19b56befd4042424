// svg_lane.hip -- lane-per-read fast path of the single-end subread-align voting step.
//
// The wave-per-read vote_kernel (svg_vote.hip) replays each read's ~30 candidates one
// at a time through the whole wavefront; at 3 Gbp that leaves it instruction-bound with
// most lanes idle.  Here every LANE owns one read, so a wave votes 64 reads at once:
//
//   gather_kernel  (thread = read x strand)  walks probe_kernel's records of its read in
//                  the reference's visiting order (subread_no, xk1, mid..last, mid-1..first;
//                  gehash_go_X, sorted-hashtable.c:984-1120), fetches the hit values and
//                  writes the read's candidate list (kv = value - offset, kP1 | offset) in a
//                  [strand][j][read] layout, so the lane kernel's j-th loads are coalesced.
//   lane_kernel    (lane = read)  per strand: init_gene_vote (gene-algorithms.h:42), the
//                  gehash_go_X tally state machine (sorted-hashtable.c:995-1107) on a per-lane
//                  vote table, then the single-end part of process_voting_junction_PE_topK
//                  (core-junction.c:2199-2530) and the SE gate of do_voting (core.c:3215-3233);
//                  finally the multi_best mapping_result_t records (core.h:350-370).
//
// Per-lane vote table.  The reference's gene_vote_t is 30 rows x 24 slots, first match
// wins in (row iix = 0,+5,-5; slot ascending) order, new slots appended to row kv/5 %30.
// Each lane keeps a pool of K <= 24 slots in LDS ([slot][lane] uint2: position, meta) with
// one singly linked list per row (heads: 30 x 5-bit fields in 5 registers, next pointer in
// the slot's meta), which visits a row's slots in exactly the reference's slot order.  The
// cold part of a slot (coverage start/end, 21-entry indel recorder) lives in a per-wave
// HBM scratch, one region per strand so that the first strand's results stay readable.
//
// A read leaves the fast path (it is appended to a deferral list and voted afterwards by
// vote_kernel, bit-identical by construction) when it needs anything this table does not
// model: more than CAP candidates on a strand, more than K slots, a shift-indel mark
// (which would trigger the reference's second voting round, sorted-hashtable.c:1016-1019),
// a read shorter than 15+gap or longer than 160 bp, or more than 31 applied subreads.
// Integer work only: no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <type_traits>
#include <string.h>
#include "subread_vote.h"
#include "svg_internal.h"
#include "svg_device.h"

#define LROWS 30
#define CW 7                 // cold words per slot: cs | rec[0] << 8, then rec[0..23] as bytes (once spilled)
#define LJW 4                // subjunc: words of a slot's subjunc_result_t (junction of the result it became)
#define LCODEW 10            // subjunc: 2-bit codes of the current strand's read text (<= 160 bases)
#define LJCW 17              // JUNCTION_CONFIRM_WINDOW (subread.h)
// per-wave cold scratch words (x 64 lanes)
#define LJLIST 24            // subjunc: minor-half candidates of a strand's results (more: the read is deferred)
__host__ __device__ constexpr int lane_cold_words(int K, bool sj, int ends = 1) { return 2 * K * CW + (sj ? 2 * K * LJW + ends * LCODEW + LJLIST : 0); }

// ---------------------------------------------------------------------------------------------
// gather: one thread per (strand, read) of a chunk
// ---------------------------------------------------------------------------------------------
struct GParams {
	const uint2 *precs;      // probe records, SoA: record q of read r at precs[q * n + r]
	const uint16_t *len;
	const uint32_t *vals;
	uint32_t n;
	int nps, gap, total_subreads, cap;
	uint32_t *cand;          // [2][cap][cs] kv
	uint16_t *cpk;           // [2][cap][cs] kP1 | off << 6
	uint16_t *ccnt;          // [2][cs] candidates, 0xffff = leave the fast path
	uint32_t cs;             // column stride of cand/cpk/ccnt
	const uint32_t *idx;     // NULL: column r = read r; else column k = read idx[k], k < min(*idx_count, cs)
	const uint32_t *idx_count;
};

__global__ void __launch_bounds__(256) gather_kernel(GParams g)
{
	const uint32_t n = g.n;
	uint32_t m = n;
	if (g.idx) { m = *g.idx_count; if (m > g.cs) m = g.cs; }
	for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < 2u * m; t += gridDim.x * 256u) {
		const uint32_t s = t >= m ? 1u : 0u, k = t - s * m;
		const uint32_t r = g.idx ? g.idx[k] : k;
		int len = g.len[r];
		if (len > SVG_READ_KEEP) len = SVG_READ_KEEP;
		const int gap = g.gap;
		uint32_t c = 0xffffu;
		if (len >= 15 + gap && len <= 160) {
			// subread offsets, core.c:3117-3171 (reads <= 160 bp)
			const int cr = (len - 15 - gap) << 16;
			int step = cr / (g.total_subreads - 1);
			if (step < (gap << 16)) step = gap << 16;
			const int applied = 1 + cr / step, np = applied * gap;
			if (applied <= 31 && np <= g.nps) {
				c = 0;
				for (int p = 0; p < np; p++) {
					const uint2 rec = g.precs[(size_t)(s * (uint32_t)g.nps + (uint32_t)p) * n + r];
					const uint32_t fwd = rec.y & 0xffffu, hits = fwd + (rec.y >> 16);
					if (!hits) continue;
					if (c + hits > (uint32_t)g.cap) { c = 0xffffu; break; }
					const int sk = p / gap, x = p - sk * gap;   // subread number, gap slot
					int off = (int)(((int64_t)step * sk) >> 16);
					if (gap > 1) off -= off % gap - x;
					const uint16_t pk = (uint16_t)((sk + 1) | (off << 6));
					for (uint32_t j = 0; j < hits; j++) {
						const uint32_t item = j < fwd ? rec.x + j : rec.x - 1u - (j - fwd);
						const size_t o = (size_t)(s * (uint32_t)g.cap + c + j) * g.cs + k;
						g.cand[o] = g.vals[item] - (uint32_t)off;
						g.cpk[o] = pk;
					}
					c += hits;
				}
			}
		}
		g.ccnt[(size_t)s * g.cs + k] = (uint16_t)c;
	}
}

// ---------------------------------------------------------------------------------------------
// lane kernel
// ---------------------------------------------------------------------------------------------
struct LParams;
// a candidate's position: the record's own word for an inline one-hit probe, else vals[item]; the
// load's index is 0 for inline ones, so a load the compiler speculates stays inside vals[]
template <class P>
__device__ __forceinline__ uint32_t lval(const P &lp, bool inl, uint32_t it)
{
	const uint32_t v = lp.vals[inl ? 0u : it];
	return inl ? it : v;
}
struct LParams {
	const uint32_t *cand;
	const uint16_t *cpk;
	const uint16_t *ccnt;
	const uint16_t *len;
	uint32_t n;
	int cap, gap, total_subreads, tol;
	uint32_t low, high;
	int multi_best, max_vote_simples, cutoff, min_votes_first, min_votes_second;
	uint8_t *out;                 // this chunk's mapping records
	uint32_t *cold;               // per-wave scratch
	uint32_t *defer_list, *defer_count;
	int defer_all;                // testing: every read takes the deferred path
	uint32_t cs;                  // column stride of cand/cpk/ccnt
	const uint32_t *idx;          // NULL: lane column r = read r; else column k = read idx[k], k < *idx_count
	const uint32_t *idx_count;    //   (columns >= cs have no candidate list and are deferred)
	const uint2 *precs;           // fused gather (NPF > 0): probe records, SoA [(end * 2 + strand) * nps + p][n]
	const uint32_t *vals;
	int nps;
	// subjunc (lane_kernel<..., SJ = true>)
	uint8_t *jout;                // subjunc_result_t records of the chunk
	uint16_t *bm_out;             // big-margin records of the chunk
	int bm_size, max_intron;
	// subjunc donor scoring on the lane (SE): read text in HBM, the .array, donor-test switches
	const char *seq, *seq2;
	const uint64_t *off, *off2;
	const uint8_t *values;
	uint32_t v_sbo, v_len, v_start, v_bytes;
	int need_donor, prefer_donor, allow_mm, rev, rev2;
	// paired-end (lane_pe_kernel)
	const uint16_t *len2;
	const uint32_t *chr_end;
	int n_chr, padding, min_pair, max_pair, mvc;
	int max_pairs;                // a pair's simples products past this go to the wave kernel (per-lane pair loop bound)
	unsigned long long *stats;    // [3] += results; [4] += deferred reads (final pass only);
	int stat_base, final_pass;    // diagnostics at stats[stat_base..+4]: deferrals by reason (3), candidates, deferrals
	// count bins (fused SE path): lane_bin_kernel lists the chunk's reads by their larger strand's
	// candidate count, bin b at bins[b * n], bin_count[b] reads; the lane kernel takes 64-read
	// groups from the heaviest bin down (NULL: lane column k = read k or idx[k])
	uint32_t *bins, *bin_count;
};

// candidate-count bins: a wave's vote loop runs as many iterations as its heaviest lane has
// candidates, so lanes of one group should carry similar counts (C3: 19 candidates per read on
// average, but the heaviest of 64 consecutive reads typically 30-40)
#define LBINS 4
__host__ __device__ constexpr int lbin_of(int c) { return c <= 8 ? 0 : (c <= 16 ? 1 : (c <= 24 ? 2 : 3)); }

// meta: votes [0,5) | last [5,10) | toli [10,15) | cursor [15,21) (6-bit signed) | next [21,27) |
// end [27] | spilled [28] | x [29,31).  votes and last (a subread number + 1) are <= 31 on this
// path (applied <= 31).  end: the slot's read end (paired-end lanes share one slot pool between
// the two tables).  spilled: the slot's indel recorder lives in the cold scratch; until its first
// indel section opens, the recorder is (first kP1, last, 0) and stays implicit.  x: the gap slot
// of the last vote, which with last gives coverage_end without a cold store per vote.
#define LM_END   (1u << 27)
#define LM_SPILL (1u << 28)
__device__ __forceinline__ int lm_votes(uint32_t m) { return (int)(m & 31u); }
__device__ __forceinline__ int lm_last(uint32_t m) { return (int)((m >> 5) & 31u); }
__device__ __forceinline__ int lm_toli(uint32_t m) { return (int)((m >> 10) & 31u); }
__device__ __forceinline__ int lm_cursor(uint32_t m) { return ((int)(m << 11)) >> 26; }
__device__ __forceinline__ uint32_t lm_next(uint32_t m) { return (m >> 21) & 63u; }
__device__ __forceinline__ int lm_x(uint32_t m) { return (int)(m >> 29); }
__device__ __forceinline__ uint32_t lm_pack(int votes, int last, int toli, int cursor, uint32_t next)
{
	return (uint32_t)votes | ((uint32_t)last << 5) | ((uint32_t)toli << 10) | (((uint32_t)cursor & 63u) << 15) | (next << 21);
}
__device__ __forceinline__ uint32_t lm_set_next(uint32_t m, uint32_t next) { return (m & ~(63u << 21)) | (next << 21); }
__device__ __forceinline__ uint32_t lm_endbit(uint32_t m) { return m & LM_END; }
// the record-side summary of a slot: spilled | last << 1 | x << 6
__device__ __forceinline__ uint32_t lm_ext(uint32_t m) { return ((m >> 28) & 1u) | ((uint32_t)lm_last(m) << 1) | ((uint32_t)lm_x(m) << 6); }
// coverage_end of a slot: the last vote's subread offset + 16 (core.c:3169-3171; sorted-hashtable.c:1046)
// the gap slot of a subread offset (off = base - base % gap + x); gap is 1 (-F) or 3 (default)
__device__ __forceinline__ int lgap_x(int off, int gap) { return gap == 1 ? 0 : (gap == 3 ? off % 3 : off % gap); }
__device__ __forceinline__ int lcov_end(int last, int x, int step, int gap)
{
	int off = (int)(((int64_t)step * (last - 1)) >> 16);
	if (gap > 1) off -= lgap_x(off, gap) - x;
	return off + 16;
}

__device__ __forceinline__ uint32_t lrow(uint32_t x) { return (x / 5u) % LROWS; }

// value selects (by-value parameters: a conditional over lvalues would select addresses and
// pin the variables to scratch)
__device__ __forceinline__ uint32_t pick(bool c, uint32_t a, uint32_t b) { return c ? a : b; }
template <typename T>
__device__ __forceinline__ T sel3(int k, T a, T b, T c) { return k == 0 ? a : (k == 1 ? b : c); }

// update_top_three (core-junction.c:908-922) with top_scores = 3, as value selects
__device__ __forceinline__ void ltop3(int &t0, int &t1, int &t2, int v)
{
	const bool g0 = v > t0, e0 = v == t0, g1 = v > t1, e1 = v == t1, g2 = v > t2;
	const bool at1 = !g0 && !e0 && g1, at2 = !g0 && !e0 && !g1 && !e1 && g2;
	const int n0 = g0 ? v : t0;
	const int n1 = g0 ? t0 : (at1 ? v : t1);
	const int n2 = (g0 || at1) ? t1 : (at2 ? v : t2);
	t0 = n0; t1 = n1; t2 = n2;
}

// 3 smallest keys, ascending (row-major slot order of one vote value)
__device__ __forceinline__ void lins3(uint32_t &a, uint32_t &b, uint32_t &c, uint32_t k)
{
	const uint32_t nc = k < b ? b : (k < c ? k : c);
	const uint32_t nb = k < a ? a : (k < b ? k : b);
	const uint32_t na = k < a ? k : a;
	a = na; b = nb; c = nc;
}

// element idx of a 3-element register "array" := val, with one select per element
#define PUT3(idx, a0, a1, a2, val) do { const int _i = (idx); const auto _v = (val); \
	a0 = _i == 0 ? _v : a0; a1 = _i == 1 ? _v : a1; a2 = _i == 2 ? _v : a2; } while (0)

template <int K, int ENDS = 1>
struct Lane {
	// row heads: 30 fields of HB bits (NIL = all ones), HPW per register, one set per end
	static constexpr int HB = K > 31 ? 6 : 5;
	static constexpr uint32_t NIL = (1u << HB) - 1u;
	static constexpr int HPW = 32 / HB, NHW = (LROWS + HPW - 1) / HPW;
	int tol;               // min(16, -I) (<= 5 on this path)
	uint32_t low;          // first valid array position
	uint2 *pm;             // LDS: pm[slot * 64 + lane] = (position, meta), halves swapped for lanes 16-31 / 48-63
	bool swp;              // this lane stores (meta, position): lane & 16
	uint32_t *cold;        // this lane's scratch: word w of slot s of strand st at cold[((st*K+s)*CW+w)*64]
	int lane;
	uint32_t h[ENDS][NHW];
	int nslots, max_vote[ENDS];
	bool dfr;
	int why;               // deferral reason (stats): 1 candidates > CAP or length, 2 slots > K, 3 shift-indel

	template <int E>
	__device__ __forceinline__ uint32_t head(uint32_t r) const
	{
		const uint32_t q = r / HPW, sh = (r - q * HPW) * HB;
		uint32_t w = h[E][0];
#pragma unroll
		for (int k = 1; k < NHW; k++) w = pick(q == (uint32_t)k, h[E][k], w);
		return (w >> sh) & NIL;
	}
	template <int E>
	__device__ __forceinline__ void set_head(uint32_t r, uint32_t s)
	{
		const uint32_t q = r / HPW, sh = (r - q * HPW) * HB;
		const uint32_t clr = ~(NIL << sh), v = s << sh;
#pragma unroll
		for (int k = 0; k < NHW; k++) h[E][k] = pick(q == (uint32_t)k, (h[E][k] & clr) | v, h[E][k]);
	}
	// The slot pool is read whole (ds_read_b64: 32-lane groups, bank (a/4) mod 64, conflict-free
	// for [slot][lane]) but its meta word is also read and written alone (ds_read_b32 /
	// ds_write_b32: bank (a/4) mod 32, so lanes l and l+16 of a group would share a bank).  Lanes
	// with bit 4 set keep the two words in the other order, which puts those 32-bit accesses of a
	// 32-lane group on 32 different banks.
	__device__ __forceinline__ uint2 slot(uint32_t s) const
	{
		const uint2 e = pm[s * 64 + lane];
		return swp ? make_uint2(e.y, e.x) : e;
	}
	__device__ __forceinline__ uint32_t meta(uint32_t s) const
	{
		return reinterpret_cast<const uint32_t *>(pm)[(s * 64 + lane) * 2 + (swp ? 0 : 1)];
	}
	__device__ __forceinline__ uint32_t spos(uint32_t s) const
	{
		return reinterpret_cast<const uint32_t *>(pm)[(s * 64 + lane) * 2 + (swp ? 1 : 0)];
	}
	__device__ __forceinline__ void set_meta(uint32_t s, uint32_t M) const
	{
		reinterpret_cast<uint32_t *>(pm)[(s * 64 + lane) * 2 + (swp ? 0 : 1)] = M;
	}
	__device__ __forceinline__ void set_slot(uint32_t s, uint32_t pos, uint32_t M) const
	{
		pm[s * 64 + lane] = swp ? make_uint2(M, pos) : make_uint2(pos, M);
	}
	__device__ __forceinline__ uint32_t *cw(int st, int s, int w) const { return cold + ((st * K + s) * CW + w) * 64; }
	// subjunc scratch after the slot words: the junction record of result slot (st, s), read codes
	__device__ __forceinline__ uint32_t *jw(int st, int s) const { return cold + (2 * K * CW + (st * K + s) * LJW) * 64; }
	__device__ __forceinline__ uint32_t *codes(int e = 0) const { return cold + (2 * K * CW + 2 * K * LJW + e * LCODEW) * 64; }
	__device__ __forceinline__ uint32_t *jlist() const { return cold + (2 * K * CW + 2 * K * LJW + ENDS * LCODEW) * 64; }
	__device__ __forceinline__ int8_t *recb(int st, int s, int i) const
	{
		return (int8_t *)cw(st, s, 1 + (i >> 2)) + (i & 3);
	}

	// init_gene_vote for every table of the lane (the slot pool is emptied)
	__device__ __forceinline__ void reset()
	{
		uint32_t all = 0;
#pragma unroll
		for (int i = 0; i < HPW; i++) all |= NIL << (i * HB);
#pragma unroll
		for (int e = 0; e < ENDS; e++) {
#pragma unroll
			for (int k = 0; k < NHW; k++) h[e][k] = all;
			max_vote[e] = 0;
		}
		nslots = 0;
	}

	// gehash_go_X body for one candidate of end E (round 0; sorted-hashtable.c:995-1107)
	template <int E>
	__device__ __forceinline__ void vote(int st, uint32_t kv, int kP1, int off, uint32_t high_b, int gap)
	{
		const uint32_t r0 = lrow(kv), rp = lrow(kv + 5u), rm = lrow(kv - 5u);
		uint32_t tail = NIL, tailM = 0;
		int ri = 0, n0 = 0;
		uint32_t s = head<E>(r0);
		bool found = false;
		for (;;) {
			while (s == NIL && ri < 2) { ri++; s = head<E>(ri == 1 ? rp : rm); }
			if (s == NIL) break;
			const uint2 e = slot(s);
			uint32_t M = e.y;
			const int d = (int)(kv - e.x);
			if (d >= -tol && d <= tol) {
				int tl = lm_toli(M), last = lm_last(M), votes = lm_votes(M);
				if (tl > 0 && d == 0) { dfr = true; why = 3; return; }   // shift-indel mark -> second round
				bool chg = false;
				if (kP1 == last && tl > 0) {   // roll-back (sorted-hashtable.c:1027-1039)
					int md = tl >= 3 ? (int)*recb(st, s, tl - 1) : 0;
					int nd = md - d;
					md -= (int)*recb(st, s, tl + 2);
					if (abs(md) > abs(nd)) { tl -= 3; last -= 1; votes -= 1; chg = true; }
				}
				if (kP1 > last) {
					votes += 1;
					int cur = lm_cursor(M);
					uint32_t spill = M & LM_SPILL;
					// coverage_end = off + 16 follows from (kP1, x) in the meta (lcov_end)
					if (d == cur) { if (spill) *recb(st, s, tl + 1) = (int8_t)kP1; }   // implicit rec[1] = last
					else {
						const int t2 = tl + 3;
						if (!spill) {
							// first indel section (tl == 0): the recorder goes to the cold scratch,
							// rec[0..7] = first kP1, last, 0, kP1, kP1, d, 0, -
							const uint32_t r0 = (*cw(st, s, 0) >> 8) & 0xffu;
							*cw(st, s, 1) = r0 | ((uint32_t)(uint8_t)last << 8) | ((uint32_t)(uint8_t)kP1 << 24);
							*cw(st, s, 2) = (uint32_t)(uint8_t)kP1 | ((uint32_t)(uint8_t)(int8_t)d << 8);
							tl = 3;
							spill = LM_SPILL;
						} else if (t2 < 21) {
							tl = t2;
							*recb(st, s, t2) = (int8_t)kP1;
							*recb(st, s, t2 + 1) = (int8_t)kP1;
							*recb(st, s, t2 + 2) = (int8_t)d;
							if (t2 < 18) *recb(st, s, t2 + 3) = 0;
						}
						cur = d;
					}
					M = lm_pack(votes, kP1, tl, cur, lm_next(M)) | lm_endbit(M) | spill | ((uint32_t)lgap_x(off, gap) << 29);
					set_meta(s, M);
					if (max_vote[E] < votes) max_vote[E] = votes;
					found = true;
					break;
				}
				if (chg) { M = lm_pack(votes, last, tl, lm_cursor(M), lm_next(M)) | (M & (LM_END | LM_SPILL | (3u << 29))); set_meta(s, M); }
			}
			if (ri == 0) { tail = s; tailM = M; n0++; }
			s = lm_next(M);
		}
		// new slot in row r0 unless it already holds GENE_VOTE_SPACE (24) slots
		if (!found && kv >= low && kv <= high_b && (K <= 24 || n0 < 24)) {
			if (nslots == K) { dfr = true; why = 2; return; }
			const uint32_t ns = (uint32_t)nslots++;
			set_slot(ns, kv, lm_pack(1, kP1, 0, 0, NIL) | (E ? LM_END : 0u) | ((uint32_t)lgap_x(off, gap) << 29));
			*cw(st, (int)ns, 0) = (uint32_t)off | ((uint32_t)kP1 << 8);   // coverage_start, rec[0] (first kP1)
			if (tail == NIL) set_head<E>(r0, ns);
			else set_meta(tail, lm_set_next(tailM, ns));
			if (max_vote[E] < 1) max_vote[E] = 1;
		}
	}
};


// mapping_result_t of a bigtable record (copy_vote_to_alignment_res, core-junction.c:1058-1071;
// indel_recorder_copy, sorted-hashtable.c:1144) from its source slot's cold state and the slot's
// record summary ext (lm_ext): coverage_end from (last, x); an unspilled recorder is
// (first kP1, last, 0)
template <class LT>
__device__ __forceinline__ void write_record(const LT &L, int src, uint32_t pos, int v, int u, uint32_t ext, int step,
                                             int gap, uint32_t (&w)[17])
{
#pragma unroll
	for (int k = 0; k < 17; k++) w[k] = 0;
	w[2] = (uint32_t)(uint16_t)v | ((uint32_t)(uint16_t)u << 16);
	if (src >= 0) {
		const int st = src >> 6, s = src & 63;
		const int lastk = (int)((ext >> 1) & 31u), xg = (int)((ext >> 6) & 7u);
		uint32_t rw[6];
		const uint32_t w0 = *L.cw(st, s, 0);
		if (ext & 1u) {
#pragma unroll
			for (int k = 0; k < 6; k++) rw[k] = *L.cw(st, s, 1 + k);
		} else {
			rw[0] = ((w0 >> 8) & 0xffu) | ((uint32_t)lastk << 8);   // rec[3] = 0 ends it
#pragma unroll
			for (int k = 1; k < 6; k++) rw[k] = 0;
		}
		const uint32_t c0w = (w0 & 0xffu) | ((uint32_t)lcov_end(lastk, xg, step, gap) << 8);
		int nrec = 0, last = 0;
#pragma unroll
		for (int t = 0; t < 7; t++) {
			const int b0 = 3 * t;
			const int k0 = (int)(int8_t)(rw[b0 >> 2] >> (8 * (b0 & 3)));
			if (nrec == 3 * t && k0 != 0) {
				nrec = 3 * t + 3;
				last = (int)(int8_t)(rw[(b0 + 2) >> 2] >> (8 * ((b0 + 2) & 3)));
			}
		}
#pragma unroll
		for (int k = 0; k < 11; k++) {
			const int i0 = 2 * k, i1 = 2 * k + 1;
			const int v0 = i0 < nrec ? (int)(int8_t)(rw[i0 >> 2] >> (8 * (i0 & 3))) : 0;
			const int v1 = i1 < nrec ? (int)(int8_t)(rw[i1 >> 2] >> (8 * (i1 & 3))) : 0;
			w[4 + k] = (uint32_t)(uint16_t)(int16_t)v0 | ((uint32_t)(uint16_t)(int16_t)v1 << 16);
		}
		w[0] = pos;
		w[1] = st ? (uint32_t)SVG_NEGATIVE_STRAND_FLAG : 0u;
		w[3] = (uint32_t)(uint8_t)(int8_t)last << 8;
		w[15] = (c0w & 0xffu) | (((c0w >> 8) & 0xffu) << 16);
	}
}

// ---------------------------------------------------------------------------------------------
// subjunc junction search on the lane (copy_vote_to_alignment_res's junction part, no fusion /
// long-del, max_insertion_at_junctions 0; reads <= 160 bp so both halves' indel offsets are 0)
// ---------------------------------------------------------------------------------------------
// base codes: A 0, G 1, C 2, T 3 (the .array's "AGCT"), 4 = 'N' past the array
#define LB_A 0
#define LB_G 1
#define LB_C 2
#define LB_T 3
__device__ __forceinline__ uint32_t labs32u(uint32_t x) { return x > 0x7fffffffu ? (0xffffffffu - x) + 1 : x; }

// gvindex_get via gvindex_get_string (gene-value-index.c:1118-1136)
__device__ __forceinline__ int lgv(const LParams &lp, uint32_t pos)
{
	const uint32_t byte = (pos - lp.v_sbo) >> 2;
	if (byte >= lp.v_bytes - 1) return 4;
	return (int)((lp.values[byte] >> ((pos & 3u) * 2u)) & 3u);
}

// is_donor_chars + paired_chars of donor_score (core-junction.c:3717-3731): GT..AG or CT..AC
__device__ __forceinline__ bool ldonor_ok(int l0, int l1, int r0, int r1)
{
	return (l0 == LB_G && l1 == LB_T && r0 == LB_A && r1 == LB_G) || (l0 == LB_C && l1 == LB_T && r0 == LB_A && r1 == LB_C);
}
__device__ __forceinline__ bool ldonor_chars(int a, int b)
{
	return (a == LB_G && b == LB_T) || (a == LB_A && b == LB_G) || (a == LB_A && b == LB_C) || (a == LB_C && b == LB_T);
}

// match_chro (gene-value-index.c:856-959, base space) over JUNCTION_CONFIRM_WINDOW bases: the read's
// 2-bit codes at `at` (rc: LCODEW words, stride 64) against the array at pos, as one 34-bit XOR
__device__ __forceinline__ int lmatch(const LParams &lp, const uint32_t *rc, int at, uint32_t pos)
{
	if ((uint32_t)(pos + LJCW) >= lp.v_len + lp.v_start) return 0;
	if (pos > 0xffff0000u) return 0;
	const uint32_t byte = (pos - lp.v_sbo) >> 2, bit = (pos & 3u) * 2u;
	if (byte >= lp.v_bytes) return 0;
	if (byte + (bit / 2 + LJCW) / 4 >= lp.v_bytes) return 0;   // the walk would hit the end
	const uint32_t *gw = (const uint32_t *)lp.values + (byte >> 2);   // the array is padded by 64 bytes
	const uint64_t g = ((uint64_t)gw[0] | ((uint64_t)gw[1] << 32)) >> ((byte & 3u) * 8u + bit);
	const int wi = at >> 4;
	const uint64_t rr = ((uint64_t)rc[wi * 64] | ((uint64_t)rc[(wi + 1) * 64] << 32)) >> ((at & 15) * 2);
	const uint64_t x = (g ^ rr) & ((1ull << (2 * LJCW)) - 1ull);
	return LJCW - __popcll((x | (x >> 1)) & 0x155555555ull);
}

// the current strand's read text as 2-bit codes (LSB-first, 16 per word) in the lane's scratch:
// strand text = the read (flip 0) or reverse_read of it (flip 1; input-files.c:1111 table, 'U' as
// 'T', anything else 'N'); match_chro counts A/G/C against 0/1/2 and every other character as T
__device__ void lcodes(const char *seq, const uint64_t *off, uint32_t r, int len, int flip, uint32_t *rc)
{
	const uint8_t *b = (const uint8_t *)(seq + off[r]);
	for (int w = 0; w < LCODEW; w++) {
		if (16 * w >= len) { rc[w * 64] = 0u; continue; }
		uint32_t acc = 0;
#pragma unroll 4   // (full unroll: 178 VGPRs, 2 waves/SIMD)
		for (int k = 0; k < 16; k++) {
			const int i = 16 * w + k;
			const int j = i < len ? (flip ? len - 1 - i : i) : 0;
			const int c = b[j];
			const uint32_t code = flip ? (c == 'A' ? 3u : c == 'C' ? 1u : c == 'G' ? 2u : (c == 'T' || c == 'U') ? 0u : 3u)
			                           : (c == 'A' ? 0u : c == 'G' ? 1u : c == 'C' ? 2u : 3u);
			acc |= (i < len ? code : 0u) << (2 * k);
		}
		rc[w * 64] = acc;
	}
}

// donor_score (core-junction.c:3675-3834) in one lane: split points mid-outward, the first strictly
// best score kept; returns the raw best score (> 0: found) with its split point and strand.  The four
// donor bases of a split point are independent loads (one round trip); the match windows follow only
// where the donor test passes.
__device__ int ldonor(const LParams &lp, const uint32_t *rc, int rl, uint32_t left, uint32_t right, int normal, int gs,
                      int ge, int &split, int &gtag)
{
	int best = -111111, dr1 = 4;   // dr1: the last fetched donor_right[1] (the reference's buffer)
	const int mid = (gs + ge) / 2, n = ge - gs;
	const uint32_t A = normal ? left : right, B = normal ? right : left;   // donor_left / donor_right sides
	for (int i = 0; i < n; i++) {
		const int sp = mid + ((i & 1) ? -((i + 1) >> 1) : ((i + 1) >> 1));
		if (sp > rl - LJCW || sp < LJCW) continue;
		const uint32_t u = (uint32_t)sp;
		const int g0 = lgv(lp, A + u), g1 = lgv(lp, A + u + 1u), g2 = lgv(lp, B + u - 2u), g3 = lgv(lp, B + u - 1u);
		bool ok = false;
		int dl0 = 4;
		if (lp.prefer_donor) {
			dl0 = g0;
			// normal: donor_right is fetched only after a donor pair on the left
			if (!normal || ldonor_chars(g0, g1)) { dr1 = g3; ok = ldonor_ok(g0, g1, g2, g3); }
		}
		if (!ok && lp.need_donor) continue;
		// (with the donor test, the default, only split points at a GT..AG / CT..AC pair get here)
		const int mLa = lmatch(lp, rc, sp - LJCW, left + u - LJCW), mLb = lmatch(lp, rc, sp, left + u);
		const int mRa = lmatch(lp, rc, sp - LJCW, right + u - LJCW), mRb = lmatch(lp, rc, sp, right + u);
		int lm, rm, ln, rn;
		if (normal) {
			lm = mLa; rm = mRb; ln = mLb; rn = mRa;
			if (lm <= LJCW - 2 || rm < 2 * LJCW - lm - lp.allow_mm || ln > LJCW - 5 || rn > LJCW - 5) continue;
		} else {
			rm = mRa; lm = mLb; rn = mRb; ln = mLa;
			if (lm + rm < 2 * LJCW - lp.allow_mm || ln > LJCW - 5 || rn > LJCW - 5) continue;
		}
		const int sc = 100 * ((ok ? 3000 : 0) + lm + rm - ln - rn);
		if (sc > best) {
			best = sc;
			split = sp;
			gtag = (dl0 == LB_G || dr1 == LB_G) ? 1 : 0;
		}
	}
	return best;
}

// (waves_per_eu 4: the subjunc variant needs 154 VGPRs unconstrained, i.e. 3 waves/SIMD; capped at
// 128 it spills 48 B/lane and the C5 lane kernel runs 3.6 -> 2.5 ms per 1M reads)
#ifndef SVG_LANE_WPE
#define SVG_LANE_WPE 4
#endif
template <int K, int NPF, bool SJ>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SVG_LANE_WPE))) lane_kernel(LParams lp)
{
	extern __shared__ __align__(16) uint8_t lds_raw[];
	const uint32_t gw = blockIdx.x, nw = gridDim.x;
	Lane<K> L;
	L.tol = lp.tol;
	L.low = lp.low;
	L.lane = (int)__lane_id();
	L.pm = reinterpret_cast<uint2 *>(lds_raw);
	L.swp = (L.lane & 16) != 0;
	L.cold = lp.cold + (size_t)gw * (lane_cold_words(K, SJ) * 64) + L.lane;
	const int mb = lp.multi_best, mvs = lp.max_vote_simples, mvf = lp.min_votes_first, mvsec = lp.min_votes_second;
	const int cutoff = lp.cutoff;
	unsigned long long nres = 0, ndef = 0, nwhy1 = 0, nwhy2 = 0, nwhy3 = 0, ncand = 0;
	const uint32_t m = lp.idx ? *lp.idx_count : lp.n;
	uint32_t bc[LBINS] = {0u, 0u, 0u, 0u}, ngroups = (m + 63u) / 64u;
	if (lp.bins) {
		ngroups = 0;
#pragma unroll
		for (int b = 0; b < LBINS; b++) { bc[b] = lp.bin_count[b]; ngroups += (bc[b] + 63u) / 64u; }
	}
	for (uint32_t g = gw; g < ngroups; g += nw) {
		uint32_t k, r;
		bool live;
		if (lp.bins) {
			// group g of the bins, heaviest bin first (the long groups start early)
			uint32_t gg = g;
			int b = LBINS - 1;
			for (; b > 0; b--) {
				const int bb = b;
				const uint32_t gb = (bc[bb] + 63u) / 64u;
				if (gg < gb) break;
				gg -= gb;
			}
			k = gg * 64u + (uint32_t)L.lane;
			live = k < bc[b];
			r = live ? lp.bins[(size_t)b * lp.n + k] : 0u;
		} else {
			k = g * 64u + (uint32_t)L.lane;
			live = k < m;
			r = !live ? 0u : lp.idx ? lp.idx[k] : k;
		}
		const bool nocol = !lp.bins && k >= lp.cs;
		L.dfr = !live || lp.defer_all || nocol;
		L.why = live && nocol ? 1 : 0;
		int len = live ? lp.len[r] : 0;
		if (len > SVG_READ_KEEP) len = SVG_READ_KEEP;
		int applied = 0, step = 0;
		if (!L.dfr && len >= 15 + lp.gap) {
			const int cr = (len - 15 - lp.gap) << 16;
			step = cr / (lp.total_subreads - 1);
			if (step < (lp.gap << 16)) step = lp.gap << 16;
			applied = 1 + cr / step;
		}
		if constexpr (NPF > 0) {
			// fused gather: the lane path's limits (the gather kernel's, for the unfused path)
			if (!L.dfr && (len < 15 + lp.gap || len > 160 || applied > 31 || applied * lp.gap > NPF || applied * lp.gap > lp.nps)) { L.dfr = true; L.why = 1; }
		}
		const uint32_t high_b = lp.high - (uint32_t)len;
		// the read's bigtable records: source (-1 none, else strand << 5 | slot), position, votes, used
		int rsrc0 = -1, rsrc1 = -1, rsrc2 = -1;
		uint32_t rpos0 = 0, rpos1 = 0, rpos2 = 0;
		int rv0 = 0, rv1 = 0, rv2 = 0, ru0 = 0, ru1 = 0, ru2 = 0;
		uint32_t rx0 = 0, rx1 = 0, rx2 = 0;   // lm_ext of the records' slots
		int nc_read = 0;
		// subjunc: the read's big-margin records (insert_big_margin_record, core-junction.c:789-811):
		// votes | start << 16 ... as (votes, start | end << 16) per record
		uint32_t bv0 = 0, bv1 = 0, bv2 = 0, bs0 = 0, bs1 = 0, bs2 = 0;
		const int nbm = SJ ? (lp.bm_size >= 3 ? lp.bm_size / 3 : 0) : 0;
		for (int st = 0; st < 2; st++) {
			if constexpr (NPF == 0) {
			const int cnt = L.dfr ? 0 : (int)lp.ccnt[(size_t)st * lp.cs + k];
			if (cnt == 0xffff) { L.dfr = true; L.why = 1; }
			const int mycnt = L.dfr ? 0 : cnt;
			nc_read += mycnt;
			L.reset();
			// ---- voting: the j-th candidates of all lanes are one coalesced load
			int mc = mycnt;
			for (int o = 32; o; o >>= 1) { int t = __shfl_xor(mc, o); mc = t > mc ? t : mc; }
			const uint32_t *cb = lp.cand + (size_t)st * lp.cap * lp.cs + k;
			const uint16_t *pb = lp.cpk + (size_t)st * lp.cap * lp.cs + k;
			uint32_t kv_a = 0, kv_b = 0;
			uint32_t pk_a = 0, pk_b = 0;
			if (0 < mycnt) { kv_a = cb[0]; pk_a = pb[0]; }
			if (1 < mycnt) { kv_b = cb[lp.cs]; pk_b = pb[lp.cs]; }
			for (int j = 0; j < mc; j++) {
				const uint32_t kv = kv_a, pk = pk_a;
				kv_a = kv_b; pk_a = pk_b;
				if (j + 2 < mycnt) { kv_b = cb[(size_t)(j + 2) * lp.cs]; pk_b = pb[(size_t)(j + 2) * lp.cs]; }
				if (j < mycnt && !L.dfr) L.template vote<0>(st, kv, (int)(pk & 63u), (int)(pk >> 6), high_b, lp.gap);
			}
			} else {
			// ---- fused gather: the read's probe records of this strand in a register window
			// (probe pb is rx[0]/ry[0]; advancing shifts the window), candidates generated in
			// the reference's visiting order (subread_no, xk1, mid..last, mid-1..first) and their
			// hit values prefetched four candidates ahead
			const int np = applied * lp.gap;
			uint32_t rx[NPF], ry[NPF];
			int cnt = 0;
#pragma unroll
			for (int p = 0; p < NPF; p++) {
				const bool ok = !L.dfr && p < np;
				const uint2 v = ok ? lp.precs[(size_t)(st * lp.nps + p) * lp.n + r] : make_uint2(0u, 0u);
				rx[p] = v.x;
				ry[p] = v.y;
				cnt += (int)((v.y & 0xffffu) + (v.y >> 16));
			}
			if (!L.dfr && cnt > lp.cap) { L.dfr = true; L.why = 1; }
			const int mycnt = L.dfr ? 0 : cnt;
			nc_read += mycnt;
			L.reset();
			int mc = mycnt;
			for (int o = 32; o; o >>= 1) { int t = __shfl_xor(mc, o); mc = t > mc ? t : mc; }
			int pb = 0;
			uint32_t jb = 0;
			auto next = [&](uint32_t &item, uint32_t &pk) __attribute__((always_inline)) -> bool {
				while (jb >= (ry[0] & 0xffffu) + (ry[0] >> 16)) {
#pragma unroll
					for (int p = 0; p + 1 < NPF; p++) { rx[p] = rx[p + 1]; ry[p] = ry[p + 1]; }
					rx[NPF - 1] = 0u;
					ry[NPF - 1] = 0u;
					pb++;
					jb = 0;
				}
				const uint32_t fwd = ry[0] & 0xffffu;
				item = jb < fwd ? rx[0] + jb : rx[0] - 1u - (jb - fwd);
				jb++;
				const int sk = lp.gap == 1 ? pb : pb / lp.gap, x = pb - sk * lp.gap;
				int off = (int)(((int64_t)step * sk) >> 16);
				if (lp.gap > 1) off -= off % lp.gap - x;
				pk = (uint32_t)(sk + 1) | ((uint32_t)off << 6);
				return false;
			};
			uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0, k0 = 0, k1 = 0, k2 = 0, k3 = 0, it = 0, pkn = 0;
			if (0 < mycnt) { q0 = lval(lp, next(it, pkn), it); k0 = pkn; }
			if (1 < mycnt) { q1 = lval(lp, next(it, pkn), it); k1 = pkn; }
			if (2 < mycnt) { q2 = lval(lp, next(it, pkn), it); k2 = pkn; }
			if (3 < mycnt) { q3 = lval(lp, next(it, pkn), it); k3 = pkn; }
			for (int j = 0; j < mc; j++) {
				const uint32_t val = q0, pk = k0;
				q0 = q1; q1 = q2; q2 = q3;
				k0 = k1; k1 = k2; k2 = k3;
				if (j + 4 < mycnt) { q3 = lval(lp, next(it, pkn), it); k3 = pkn; }
				if (j < mycnt && !L.dfr) L.template vote<0>(st, val - (pk >> 6), (int)(pk & 63u), (int)(pk >> 6), high_b, lp.gap);
			}
			}
			if (L.dfr) continue;
			// ---- SE gate (core.c:3215-3233) and top-K (core-junction.c:2199-2530, ends = 1)
			if (L.max_vote[0] >= mvf) {
				int t0 = 0, t1 = 0, t2 = 0;
				for (int s = 0; s < L.nslots; s++) ltop3(t0, t1, t2, lm_votes(L.meta(s)));
				if (rv0 > 0) ltop3(t0, t1, t2, rv0);
				if (mb > 1 && rv1 > 0) ltop3(t0, t1, t2, rv1);
				if (mb > 2 && rv2 > 0) ltop3(t0, t1, t2, rv2);
				const bool ok0 = t0 >= 1, ok1 = ok0 && t1 >= 1 && t0 - t1 <= cutoff, ok2 = ok1 && t2 >= 1 && t0 - t2 <= cutoff;
				if constexpr (SJ) {
					// big-margin records: every slot the first value's row-major scan visits before
					// max_vote_simples slots of that value are taken (core-junction.c:2276-2277)
					if (ok0 && nbm > 0) {
						int taken = 0;
						for (uint32_t row = 0; row < LROWS && taken < mvs; row++) {
							uint32_t q = L.template head<0>(row);
							while (q != Lane<K>::NIL && taken < mvs) {
								const uint32_t M = L.meta(q);
								const int v = lm_votes(M);
								if (v >= t2) {
									const int rs = (int)(*L.cw(st, (int)q, 0) & 0xffu);
									const int re = lcov_end(lm_last(M), lm_x(M), step, lp.gap);
									const uint32_t vv = (uint32_t)(v & 255);
									const uint32_t se = st ? ((uint32_t)(uint16_t)(len - re) | ((uint32_t)(uint16_t)(len - rs) << 16))
									                       : ((uint32_t)rs | ((uint32_t)re << 16));
									const int x1 = vv >= bv0 ? 0 : (nbm > 1 && vv >= bv1) ? 1 : (nbm > 2 && vv >= bv2) ? 2 : 3;
									if (x1 < nbm) {
										if (x1 <= 1 && nbm > 2) { bv2 = bv1; bs2 = bs1; }
										if (x1 == 0 && nbm > 1) { bv1 = bv0; bs1 = bs0; }
										PUT3(x1, bv0, bv1, bv2, vv);
										PUT3(x1, bs0, bs1, bs2, se);
									}
								}
								if (v == t0 && v >= mvsec) taken++;
								q = lm_next(M);
							}
						}
					}
				}
				// table slots of each value in row-major order (row, then slot order = pool order)
				uint32_t a0 = ~0u, b0 = ~0u, c0 = ~0u, a1 = ~0u, b1 = ~0u, c1 = ~0u, a2 = ~0u, b2 = ~0u, c2 = ~0u;
				for (int s = 0; s < L.nslots; s++) {
					const uint2 e = L.slot(s);
					const int v = lm_votes(e.y);
					if (v < mvsec) continue;
					const uint32_t key = (lrow(e.x) << 6) | (uint32_t)s;
					if (ok0 && v == t0) lins3(a0, b0, c0, key);
					else if (ok1 && v == t1) lins3(a1, b1, c1, key);
					else if (ok2 && v == t2) lins3(a2, b2, c2, key);
				}
				// simples (simple_mapping_t), in the reference's order; src: slot | 64, or stored index
				int ns = 0;
				int sv0 = 0, sv1 = 0, sv2 = 0, sk0 = 0, sk1 = 0, sk2 = 0;
				uint32_t sp0 = 0, sp1 = 0, sp2 = 0;
				auto add = [&](int kind, uint32_t pos, int v) __attribute__((always_inline)) {
					PUT3(ns, sk0, sk1, sk2, kind);
					PUT3(ns, sp0, sp1, sp2, pos);
					PUT3(ns, sv0, sv1, sv2, v);
					ns++;
				};
				auto add_val = [&](int N, uint32_t ka, uint32_t kb, uint32_t kc) __attribute__((always_inline)) {
					if (ka != ~0u && ns < mvs) add(128 | (int)(ka & 63u), L.spos((ka & 63u)), N);
					if (kb != ~0u && ns < mvs) add(128 | (int)(kb & 63u), L.spos((kb & 63u)), N);
					if (kc != ~0u && ns < mvs) add(128 | (int)(kc & 63u), L.spos((kc & 63u)), N);
					if (ns < mvs && rv0 == N) add(0, rpos0, N);
					if (mb > 1 && ns < mvs && rv1 == N) add(1, rpos1, N);
					if (mb > 2 && ns < mvs && rv2 == N) add(2, rpos2, N);
				};
				if (ok0) add_val(t0, a0, b0, c0);
				if (ok1 && ns < mvs) add_val(t1, a1, b1, c1);
				if (ok2 && ns < mvs) add_val(t2, a2, b2, c2);
				// single-end results: simples with >= min_votes_first votes, distinct positions
				int cur = 0;
				int ts0 = -1, ts1 = -1, ts2 = -1, tu0 = 0, tu1 = 0, tu2 = 0, tv0 = 0, tv1 = 0, tv2 = 0;
				uint32_t tp0 = 0, tp1 = 0, tp2 = 0, tx0 = 0, tx1 = 0, tx2 = 0;
				auto emit = [&](int kind, uint32_t pos, int v) __attribute__((always_inline)) {
					if (cur >= mb || v < mvf) return;
					if ((cur > 0 && tp0 == pos) || (cur > 1 && tp1 == pos)) return;
					int src, u, vv = v;
					uint32_t x;
					if (kind & 128) { src = (st << 6) | (kind & 63); u = applied; x = lm_ext(L.meta((kind & 63))); }
					else {
						src = sel3(kind, rsrc0, rsrc1, rsrc2);
						u = sel3(kind, ru0, ru1, ru2);
						pos = sel3(kind, rpos0, rpos1, rpos2);
						vv = sel3(kind, rv0, rv1, rv2);
						x = sel3(kind, rx0, rx1, rx2);
					}
					PUT3(cur, tx0, tx1, tx2, x);
					PUT3(cur, ts0, ts1, ts2, src);
					PUT3(cur, tp0, tp1, tp2, pos);
					PUT3(cur, tv0, tv1, tv2, vv);
					PUT3(cur, tu0, tu1, tu2, u);
					cur++;
				};
				if (ns > 0) emit(sk0, sp0, sv0);
				if (ns > 1) emit(sk1, sp1, sv1);
				if (ns > 2) emit(sk2, sp2, sv2);
				if constexpr (SJ) {
					// junction part of copy_vote_to_alignment_res (core-junction.c:1073-1334) for each
					// result taken from this table: every other slot, in the table's row-major order, is
					// a minor-half candidate -- test_junction_minor, the overlap / distance tests,
					// is_better_inner (core-junction.c:961) against the minor kept so far, then
					// donor_score.  The junction record goes to the result slot's scratch; the result's
					// ext carries bit 12 (record present) and the result_flags bits 0-1 (bits 13-14)
					// phase 1: the candidates that pass the J-independent tests, per result in row-major
					// order, into the lane's list (c << 6 | slot)
					uint32_t *lst = L.jlist();
					int nl = 0;
					for (int c = 0; c < cur && !L.dfr; c++) {
						const int src = sel3(c, ts0, ts1, ts2);
						if (src < 0 || (src >> 6) != st) continue;
						const int sM = src & 63;
						const uint2 eM = L.slot(sM);
						const int vM = lm_votes(eM.y);
						const int csM = (int)(*L.cw(st, sM, 0) & 0xffu), ceM = lcov_end(lm_last(eM.y), lm_x(eM.y), step, lp.gap);
						for (uint32_t row = 0; row < LROWS && !L.dfr; row++) {
							uint32_t q = L.template head<0>(row);
							while (q != Lane<K>::NIL) {
								const uint2 e2 = L.slot(q);
								const uint32_t qs = q;
								q = lm_next(e2.y);
								if ((int)qs == sM || vM < lm_votes(e2.y)) continue;
								const long long dist = (long long)eM.x - (long long)e2.x;
								if ((dist < 0 ? -dist : dist) > (long long)lp.max_intron) continue;
								const int cs2 = (int)(*L.cw(st, (int)qs, 0) & 0xffu), ce2 = lcov_end(lm_last(e2.y), lm_x(e2.y), step, lp.gap);
								if (csM == cs2 || ceM == ce2) continue;
								if (csM > cs2 ? eM.x < e2.x : eM.x > e2.x) continue;   // test_junction_minor
								const int ov = csM > cs2 ? ce2 - csM : ceM - cs2;
								if (ov > 14 || abs((int)dist) < 6) continue;
								if (nl == LJLIST) { L.dfr = true; L.why = 2; break; }
								lst[nl * 64] = ((uint32_t)c << 6) | qs;
								nl++;
							}
						}
					}
					if (L.dfr) continue;
					// phase 2: every lane walks its list at the same step k, so the wave scores its
					// lanes' candidates together: is_better_inner against the minor kept so far for
					// that result, then donor_score
					if (nl > 0) lcodes(lp.seq, lp.off, r, len, st ^ lp.rev, L.codes());
					int Jc = -1, Jv = 0, Jcs = 0, Jce = 0, Jsplit = 0, Jnormal = 0, Jf = -1;
					uint32_t Jpos = 0, Mpos = 0;
					int Mcs = 0, Mce = 0, sM = 0;
					auto flush = [&]() __attribute__((always_inline)) {
						if (Jf < 0) return;
						uint32_t *jw = L.jw(st, sM);
						jw[0] = (uint32_t)(uint16_t)Jsplit | ((uint32_t)(uint16_t)Jv << 16);
						jw[64] = ((uint32_t)(Jnormal ? 0 : 1) << 16) | ((uint32_t)(Jnormal ? 1 : 0) << 24);
						jw[128] = Jpos;
						jw[192] = (uint32_t)(uint16_t)Jcs | ((uint32_t)(uint16_t)Jce << 16);
						PUT3(Jc, tx0, tx1, tx2, sel3(Jc, tx0, tx1, tx2) | (1u << 12) | ((uint32_t)Jf << 13));
					};
					for (int k = 0; k < nl; k++) {
						const uint32_t ent = lst[k * 64];
						const int c = (int)(ent >> 6), qs = (int)(ent & 63u);
						if (c != Jc) {
							flush();
							Jc = c; Jv = 0; Jcs = 0; Jce = 0; Jsplit = 0; Jnormal = 0; Jf = -1; Jpos = 0;
							sM = sel3(c, ts0, ts1, ts2) & 63;
							const uint2 eM = L.slot(sM);
							Mpos = eM.x;
							Mcs = (int)(*L.cw(st, sM, 0) & 0xffu);
							Mce = lcov_end(lm_last(eM.y), lm_x(eM.y), step, lp.gap);
						}
						const uint2 e2 = L.slot(qs);
						const int V = lm_votes(e2.y);
						const int cs2 = (int)(*L.cw(st, qs, 0) & 0xffu), ce2 = lcov_end(lm_last(e2.y), lm_x(e2.y), step, lp.gap);
						// is_better_inner (core-junction.c:961)
						const int oldi = (int)labs32u(Mpos - Jpos), intr = (int)labs32u(Mpos - e2.x);
						const int cl = ce2 - cs2, jl = Jce - Jcs;
						if (!(V > Jv || (V == Jv && cl > jl) || (V == Jv && cl == jl && intr < oldi))) continue;
						const int gs = Mcs > cs2 ? ce2 - 8 : Mce - 8;
						const int ge = Mcs < cs2 ? cs2 + 8 : Mcs + 8;
						const int normal = 1 != (int)(Mcs > cs2) + (int)(Mpos > e2.x);
						int split = 0, gtag = 0;
						const int best = ldonor(lp, L.codes(), len, Mpos < e2.x ? Mpos : e2.x, Mpos > e2.x ? Mpos : e2.x, normal,
						                        gs > 0 ? gs : 0, ge < len ? ge : len, split, gtag);
						if (best > 0) {
							Jpos = e2.x; Jv = V; Jcs = cs2; Jce = ce2; Jsplit = split; Jnormal = normal;
							Jf = best < 290000 ? 3 : (gtag ? 1 : 0);   // is_donor_found_or_annotation, GT/AG strand
						}
					}
					flush();
				}
				if (cur > 0) { rsrc0 = ts0; rpos0 = tp0; rv0 = tv0; ru0 = tu0; rx0 = tx0; } else rv0 = 0;
				if (cur > 1) { rsrc1 = ts1; rpos1 = tp1; rv1 = tv1; ru1 = tu1; rx1 = tx1; } else rv1 = 0;
				if (cur > 2) { rsrc2 = ts2; rpos2 = tp2; rv2 = tv2; ru2 = tu2; rx2 = tx2; } else rv2 = 0;
			} else if (rv0 < 1) {
				if (applied > ru0) ru0 = applied;   // used_subreads_in_vote (noninformative stays 0)
			}
		}
		if (!L.dfr) ncand += (unsigned long long)nc_read;
		if constexpr (SJ) {
			if (!L.dfr && lp.bm_out) {
				uint16_t *bd = lp.bm_out + (size_t)r * SVG_BIG_MARGIN_WORDS;
				const uint32_t bvv[3] = {bv0, bv1, bv2}, bss[3] = {bs0, bs1, bs2};
#pragma unroll
				for (int k = 0; k < 3; k++) {
					bd[3 * k] = (uint16_t)bvv[k];
					bd[3 * k + 1] = (uint16_t)(bss[k] & 0xffffu);
					bd[3 * k + 2] = (uint16_t)(bss[k] >> 16);
				}
			}
		}
		// ---- the read's multi_best records (copy_vote_to_alignment_res, core-junction.c:1058-1071;
		// indel_recorder_copy, sorted-hashtable.c:1144)
		if (!L.dfr) {
			uint32_t *dst = (uint32_t *)(lp.out + (size_t)r * mb * 68);
			for (int i = 0; i < mb; i++) {
				const int src = sel3(i, rsrc0, rsrc1, rsrc2);
				const uint32_t pos = sel3(i, rpos0, rpos1, rpos2);
				const int v = sel3(i, rv0, rv1, rv2);
				const int u = sel3(i, ru0, ru1, ru2);
				uint32_t w[17];
				const uint32_t x = sel3(i, rx0, rx1, rx2);
				write_record(L, src, pos, v, u, x, step, lp.gap, w);
				if constexpr (SJ) {
					// the result's subjunc_result_t (empty without a minor half); a zero-vote record
					// keeps the stale one with minor_votes 0 (topk's reset of unused results)
					uint4 jr = make_uint4(0u, 0u, 0u, 0u);
					if (src >= 0 && ((x >> 12) & 1u)) {
						const uint32_t *jw = L.jw(src >> 6, src & 63);
						jr = make_uint4(v > 0 ? jw[0] : (jw[0] & 0xffffu), jw[64], jw[128], jw[192]);
						w[1] |= (x >> 13) & 3u;
					}
					*(uint4 *)(lp.jout + ((size_t)r * mb + i) * 16) = jr;
				}
#pragma unroll
				for (int k = 0; k < 17; k++) dst[i * 17 + k] = w[k];
				nres += v > 0;
			}
		}
		// ---- deferred reads: one atomic per wave
		const unsigned long long dm = __ballot(L.dfr && live);
		if (dm) {
			uint32_t base = 0;
			const int leader = __ffsll((long long)dm) - 1;
			if (L.lane == leader) base = atomicAdd(lp.defer_count, (uint32_t)__popcll(dm));
			base = __shfl(base, leader);
			if (L.dfr && live) lp.defer_list[base + __popcll(dm & ((1ull << L.lane) - 1ull))] = r;
			ndef += (unsigned long long)__popcll(dm);
		}
		if (lp.stats) {
			nwhy1 += (unsigned long long)__popcll(__ballot(L.dfr && live && L.why == 1));
			nwhy2 += (unsigned long long)__popcll(__ballot(L.dfr && live && L.why == 2));
			nwhy3 += (unsigned long long)__popcll(__ballot(L.dfr && live && L.why == 3));
		}
	}
	if (lp.stats) {
		for (int o = 32; o; o >>= 1) { nres += __shfl_xor(nres, o); ncand += __shfl_xor(ncand, o); }
		if (L.lane == 0) {
			atomicAdd(&lp.stats[3], nres);
			if (lp.final_pass) atomicAdd(&lp.stats[4], ndef);
			// diagnostics (svg_debug_counters): deferrals by reason, candidates voted, deferrals
			unsigned long long *d = lp.stats + lp.stat_base;
			atomicAdd(&d[0], nwhy1);
			atomicAdd(&d[1], nwhy2);
			atomicAdd(&d[2], nwhy3);
			atomicAdd(&d[3], ncand);
			atomicAdd(&d[4], ndef);
		}
	}
}


// ---------------------------------------------------------------------------------------------
// paired-end lane kernel: one lane per read pair
// ---------------------------------------------------------------------------------------------
// locate_gene_position_max(..., NULL, NULL, rl = 0), gene-algorithms.c:441-511
__device__ __forceinline__ int llocate(const uint32_t *ce, int ntot, int padding, uint32_t linear, int &chr, int &pos)
{
	int lo = 0, hi = ntot, n;
	chr = -1;
	pos = -1;
	for (;;) {
		if (hi <= lo + 1) { n = lo - 2 > 0 ? lo - 2 : 0; break; }
		const int mid = (lo + hi) / 2;
		if (ce[mid] > linear) hi = mid; else lo = mid + 1;
	}
	for (; n < ntot; n++) {
		const uint32_t c = ce[n];
		if (c > linear) {
			pos = n == 0 ? (int)linear : (int)(linear - ce[n - 1]);
			if (linear > c + 15u - (uint32_t)padding) return 1;
			if (pos < padding) return 1;
			pos -= padding;
			chr = n;
			return 0;
		}
	}
	return -1;
}

#ifndef LANE_PE_K
#define LANE_PE_K 31   // shared by both ends' tables (<= 47: 6-bit ids, stored results at LPE_RID + i)
#endif
// simples (simple_mapping_t) of one end as a packed list of 6-bit ids: slot (< LPE_RID) or
// LPE_RID + stored index; PLW words hold 5 * PLW >= LANE_PE_K slots + 3 stored records
#define PLW ((LANE_PE_K + 3 + 4) / 5)
__device__ __forceinline__ uint32_t pl_get(const uint32_t (&w)[PLW], int i)
{
	const int q = i / 5, sh = (i - q * 5) * 6;
	uint32_t x = w[0];
#pragma unroll
	for (int k = 1; k < PLW; k++) x = pick(q == k, w[k], x);
	return (x >> sh) & 63u;
}
__device__ __forceinline__ void pl_put(uint32_t (&w)[PLW], int i, uint32_t id)
{
	const int q = i / 5, sh = (i - q * 5) * 6;
#pragma unroll
	for (int k = 0; k < PLW; k++) w[k] = pick(q == k, w[k] | (id << sh), w[k]);
}

// a record of the read's bigtable: rm = (src + 1) | votes << 8 | used << 16 (src = strand << 6 | slot,
// 0 = none), rp = selected_position
#define RM(src, v, u) ((uint32_t)((src) + 1) | ((uint32_t)(v) << 8) | ((uint32_t)(u) << 16))
#define RM_SRC(m) ((int)((m) & 255u) - 1)
#define RM_V(m) ((int)(((m) >> 8) & 255u))
#define RM_U(m) ((int)(((m) >> 16) & 63u))
#define RM_EXT(m) ((m) >> 22)          // lm_ext of the record's slot, above used (<= 31)
#define RM_SETV(m, v) (((m) & ~(255u << 8)) | ((uint32_t)(v) << 8))

// SJ: subjunc pairs (process_voting_junction_PE_topK with copy_vote's junction part): big-margin
// records per end and the junction search / donor scoring of every record taken from a table, as
// in lane_kernel
// (waves_per_eu 3: the subjunc variant needs 179 VGPRs unconstrained, 168 without spills at 3 waves)
// simples of a pair: slot ids < LPE_RID, the end's stored results (multi-block) at LPE_RID + i (6-bit ids)
#define LPE_RID 48u
template <int K, int NPF, bool SJ>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) lane_pe_kernel(LParams lp)
{
	extern __shared__ __align__(16) uint8_t lds_raw[];
	const uint32_t gw = blockIdx.x, nw = gridDim.x;
	Lane<K, 2> L;
	L.tol = lp.tol;
	L.low = lp.low;
	L.lane = (int)__lane_id();
	L.pm = reinterpret_cast<uint2 *>(lds_raw);
	L.swp = (L.lane & 16) != 0;
	L.cold = lp.cold + (size_t)gw * (lane_cold_words(K, SJ, 2) * 64) + L.lane;
	const int mb = lp.multi_best, mvs = lp.max_vote_simples, mvf = lp.min_votes_first, mvsec = lp.min_votes_second;
	const int cutoff = lp.cutoff, mvc = lp.mvc;
	unsigned long long nres = 0, ndef = 0, nwhy1 = 0, nwhy2 = 0, nwhy3 = 0, ncand = 0;
	for (uint32_t g0 = gw * 64u; g0 < lp.n; g0 += nw * 64u) {
		const uint32_t r = g0 + (uint32_t)L.lane;
		const bool live = r < lp.n;
		L.dfr = !live || lp.defer_all;
		L.why = 0;
		int len[2], applied[2], step[2];
		uint32_t high_b[2];
#pragma unroll
		for (int e = 0; e < 2; e++) {
			int l = live ? (e ? lp.len2[r] : lp.len[r]) : 0;
			if (l > SVG_READ_KEEP) l = SVG_READ_KEEP;
			len[e] = l;
			applied[e] = 0;
			step[e] = 0;
			if (l >= 15 + lp.gap) {
				const int cr = (l - 15 - lp.gap) << 16;
				step[e] = cr / (lp.total_subreads - 1);
				if (step[e] < (lp.gap << 16)) step[e] = lp.gap << 16;
				applied[e] = 1 + cr / step[e];
			}
			if (!L.dfr && (l < 15 + lp.gap || l > 160 || applied[e] > 31 || applied[e] * lp.gap > NPF || applied[e] * lp.gap > lp.nps)) { L.dfr = true; L.why = 1; }
			high_b[e] = lp.high - (uint32_t)l;
		}
		// bigtable records of both ends
		uint32_t rm0[3] = {0, 0, 0}, rm1[3] = {0, 0, 0}, rp0[3] = {0, 0, 0}, rp1[3] = {0, 0, 0};
		// subjunc: big-margin records of each end, (votes, start | end << 16)
		uint32_t bv[2][3] = {{0, 0, 0}, {0, 0, 0}}, bs[2][3] = {{0, 0, 0}, {0, 0, 0}};
		const int nbm = SJ ? (lp.bm_size >= 3 ? lp.bm_size / 3 : 0) : 0;
		int nc_read = 0;
		// subjunc: a nibble per (end, record) at (end * 3 + i) * 4: bit 0 = the record has a junction
		// record in the scratch of its slot, bits 1-2 = its result_flags bits 0-1
		uint32_t jm = 0;
		for (int st = 0; st < 2; st++) {
			L.reset();
			// ---- both ends' tables: fused gather as in lane_kernel, records of (end, strand)
			auto vote_end = [&](auto E_) __attribute__((always_inline)) {
				constexpr int E = decltype(E_)::value;
				const int np = applied[E] * lp.gap;
				uint32_t rx[NPF], ry[NPF];
				int cnt = 0;
#pragma unroll
				for (int p = 0; p < NPF; p++) {
					const bool ok = !L.dfr && p < np;
					const uint2 v = ok ? lp.precs[(size_t)((E * 2 + st) * lp.nps + p) * lp.n + r] : make_uint2(0u, 0u);
					rx[p] = v.x;
					ry[p] = v.y;
					cnt += (int)((v.y & 0xffffu) + (v.y >> 16));
				}
				if (!L.dfr && cnt > lp.cap) { L.dfr = true; L.why = 1; }
				const int mycnt = L.dfr ? 0 : cnt;
				nc_read += mycnt;
				int mc = mycnt;
				for (int o = 32; o; o >>= 1) { int t = __shfl_xor(mc, o); mc = t > mc ? t : mc; }
				int pb = 0;
				uint32_t jb = 0;
				auto next = [&](uint32_t &item, uint32_t &pk) __attribute__((always_inline)) -> bool {
					while (jb >= (ry[0] & 0xffffu) + (ry[0] >> 16)) {
#pragma unroll
						for (int p = 0; p + 1 < NPF; p++) { rx[p] = rx[p + 1]; ry[p] = ry[p + 1]; }
						rx[NPF - 1] = 0u;
						ry[NPF - 1] = 0u;
						pb++;
						jb = 0;
					}
					const uint32_t fwd = ry[0] & 0xffffu;
					item = jb < fwd ? rx[0] + jb : rx[0] - 1u - (jb - fwd);
					jb++;
					const int sk = lp.gap == 1 ? pb : pb / lp.gap, x = pb - sk * lp.gap;
					int off = (int)(((int64_t)step[E] * sk) >> 16);
					if (lp.gap > 1) off -= off % lp.gap - x;
					pk = (uint32_t)(sk + 1) | ((uint32_t)off << 6);
					return false;
				};
				uint32_t q0 = 0, q1 = 0, q2 = 0, q3 = 0, k0 = 0, k1 = 0, k2 = 0, k3 = 0, it = 0, pkn = 0;
				if (0 < mycnt) { q0 = lval(lp, next(it, pkn), it); k0 = pkn; }
				if (1 < mycnt) { q1 = lval(lp, next(it, pkn), it); k1 = pkn; }
				if (2 < mycnt) { q2 = lval(lp, next(it, pkn), it); k2 = pkn; }
				if (3 < mycnt) { q3 = lval(lp, next(it, pkn), it); k3 = pkn; }
				for (int j = 0; j < mc; j++) {
					const uint32_t val = q0, pk = k0;
					q0 = q1; q1 = q2; q2 = q3;
					k0 = k1; k1 = k2; k2 = k3;
					if (j + 4 < mycnt) { q3 = lval(lp, next(it, pkn), it); k3 = pkn; }
					if (j < mycnt && !L.dfr) L.template vote<E>(st, val - (pk >> 6), (int)(pk & 63u), (int)(pk >> 6), high_b[E], lp.gap);
				}
			};
			vote_end(std::integral_constant<int, 0>());
			vote_end(std::integral_constant<int, 1>());
			if (L.dfr) continue;
			// ---- process_voting_junction_PE_topK (core-junction.c:2199-2530), ends = 2
			// (1) top-3 distinct vote values per end over its table and stored records
			int ta[2][3];
#pragma unroll
			for (int e = 0; e < 2; e++) { ta[e][0] = 0; ta[e][1] = 0; ta[e][2] = 0; }
			for (int s = 0; s < L.nslots; s++) {
				const uint32_t M = L.meta(s);
				const int v = lm_votes(M);
				if (lm_endbit(M)) ltop3(ta[1][0], ta[1][1], ta[1][2], v);
				else ltop3(ta[0][0], ta[0][1], ta[0][2], v);
			}
#pragma unroll
			for (int i = 0; i < 3; i++) {
				if (i < mb && RM_V(rm0[i]) > 0) ltop3(ta[0][0], ta[0][1], ta[0][2], RM_V(rm0[i]));
				if (i < mb && RM_V(rm1[i]) > 0) ltop3(ta[1][0], ta[1][1], ta[1][2], RM_V(rm1[i]));
			}
			// (2) simples per end, in the reference's order: per vote value, the table's slots in
			// row-major order, then the stored records of that value
			uint32_t pl[2][PLW];
			static_assert(5 * PLW >= K + 3, "simples list too short for the slot pool");
			int ns[2] = {0, 0};
			auto simples = [&](auto E_) __attribute__((always_inline)) {
				constexpr int E = decltype(E_)::value;
#pragma unroll
				for (int k = 0; k < PLW; k++) pl[E][k] = 0;
#pragma unroll
				for (int tk = 0; tk < 3; tk++) {
					const int N = ta[E][tk];
					if (ns[E] >= mvs || N < 1 || ta[E][0] - N > cutoff) break;
					if (SJ && tk == 0 && nbm > 0) {
						// the first value's row-major scan, up to max_vote_simples simples: every slot it
						// visits with votes >= the third top value is a big-margin record
						// (core-junction.c:2276-2277; insert_big_margin_record :789-811)
						for (uint32_t row = 0; row < LROWS && ns[E] < mvs; row++) {
							uint32_t s = L.template head<E>(row);
							while (s != Lane<K, 2>::NIL && ns[E] < mvs) {
								const uint32_t M = L.meta(s);
								const int v = lm_votes(M);
								if (v >= ta[E][2]) {
									const int rs = (int)(*L.cw(st, (int)s, 0) & 0xffu);
									const int re = lcov_end(lm_last(M), lm_x(M), step[E], lp.gap);
									const uint32_t vv = (uint32_t)(v & 255);
									const uint32_t se = st ? ((uint32_t)(uint16_t)(len[E] - re) | ((uint32_t)(uint16_t)(len[E] - rs) << 16))
									                       : ((uint32_t)rs | ((uint32_t)re << 16));
									const int x1 = vv >= bv[E][0] ? 0 : (nbm > 1 && vv >= bv[E][1]) ? 1 : (nbm > 2 && vv >= bv[E][2]) ? 2 : 3;
									if (x1 < nbm) {
										if (x1 <= 1 && nbm > 2) { bv[E][2] = bv[E][1]; bs[E][2] = bs[E][1]; }
										if (x1 == 0 && nbm > 1) { bv[E][1] = bv[E][0]; bs[E][1] = bs[E][0]; }
										PUT3(x1, bv[E][0], bv[E][1], bv[E][2], vv);
										PUT3(x1, bs[E][0], bs[E][1], bs[E][2], se);
									}
								}
								if (v == N && N >= mvsec) { pl_put(pl[E], ns[E], s); ns[E]++; }
								s = lm_next(M);
							}
						}
					} else if (N >= mvsec) {
						for (uint32_t row = 0; row < LROWS; row++) {
							uint32_t s = L.template head<E>(row);
							while (s != Lane<K, 2>::NIL) {
								const uint32_t M = L.meta(s);
								if (lm_votes(M) == N && ns[E] < mvs) { pl_put(pl[E], ns[E], s); ns[E]++; }
								s = lm_next(M);
							}
						}
					}
#pragma unroll
					for (int i = 0; i < 3; i++) {
						const uint32_t m = E ? rm1[i] : rm0[i];
						if (i < mb && ns[E] < mvs && RM_V(m) == N) { pl_put(pl[E], ns[E], LPE_RID + (uint32_t)i); ns[E]++; }
					}
				}
			};
			simples(std::integral_constant<int, 0>());
			simples(std::integral_constant<int, 1>());
			if (ns[0] * ns[1] > lp.max_pairs) { L.dfr = true; L.why = 2; continue; }   // bounded per-lane pair loop
			// value / position / record of a simple
			auto sv = [&](int E, uint32_t id, uint32_t &pos) __attribute__((always_inline)) -> int {
				if (id < LPE_RID) { const uint2 x = L.slot(id); pos = x.x; return lm_votes(x.y); }
				const int i = (int)id - (int)LPE_RID;
				const uint32_t m = E ? sel3(i, rm1[0], rm1[1], rm1[2]) : sel3(i, rm0[0], rm0[1], rm0[2]);
				pos = E ? sel3(i, rp1[0], rp1[1], rp1[2]) : sel3(i, rp0[0], rp0[1], rp0[2]);
				return RM_V(m);
			};
			// (3) pair scores into the comb buffer (<= max_vote_combinations, first come first kept on ties)
			int ncomb = 0;
			uint32_t ca0 = 0, ca1 = 0, ca2 = 0, cb0 = 0, cb1 = 0, cb2 = 0;
			int cs0 = 0, cs1 = 0, cs2 = 0;
			for (int i = 0; i < ns[0]; i++) {
				const uint32_t ida = pl_get(pl[0], i);
				uint32_t pa;
				const int va = sv(0, ida, pa);
				int c1 = -1, q1 = -1;
				const int e1 = llocate(lp.chr_end, lp.n_chr, lp.padding, pa, c1, q1);
				for (int j = 0; j < ns[1]; j++) {
					const uint32_t idb = pl_get(pl[1], j);
					uint32_t pb2;
					const int vb = sv(1, idb, pb2);
					if ((va > vb ? va : vb) < mvf) continue;
					int c2 = -1, q2 = -1;
					const int e2 = llocate(lp.chr_end, lp.n_chr, lp.padding, pb2, c2, q2);
					bool pe = false, same = false;
					if (e1 == 0 && e2 == 0) {   // test_PE_and_same_chro, core.c:4819-4845
						long long tl = (long long)q1 - q2;
						tl = abs((int)tl);
						tl += (q1 > q2) ? len[0] : len[1];
						const uint32_t tli = (uint32_t)tl;
						if (c1 == c2) {
							same = true;
							if (tli >= (uint32_t)lp.min_pair && tli <= (uint32_t)lp.max_pair) pe = true;
						}
					}
					if (!pe && (va < vb ? va : vb) < mvf) continue;
					const int sc = (va + vb) * (pe ? 1300 : (same ? 1000 : 800));
					const int t = (ncomb > 0 && cs0 >= sc) + (ncomb > 1 && cs1 >= sc) + (ncomb > 2 && cs2 >= sc);
					if (t < mvc) {
						// shift entries t.. down by one (the last falls off), insert at t
						if (t <= 1 && mvc > 2) { ca2 = ca1; cb2 = cb1; cs2 = cs1; }
						if (t == 0 && mvc > 1) { ca1 = ca0; cb1 = cb0; cs1 = cs0; }
						PUT3(t, ca0, ca1, ca2, ida);
						PUT3(t, cb0, cb1, cb2, idb);
						PUT3(t, cs0, cs1, cs2, sc);
						if (ncomb < mvc) ncomb++;
					}
				}
			}
			// (4) results of each end
			uint32_t tm0[3] = {0, 0, 0}, tm1[3] = {0, 0, 0}, tp0[3] = {0, 0, 0}, tp1[3] = {0, 0, 0};
			int cur[2] = {0, 0};
			uint32_t tjm = 0, needj = 0;   // subjunc: the new records' nibbles; records needing a junction search
			auto emit = [&](int E, uint32_t id) __attribute__((always_inline)) {
				uint32_t pos;
				const int v = sv(E, id, pos);
				uint32_t m;
				if (id < LPE_RID) m = RM((st << 6) | (int)id, v, applied[E]) | (lm_ext(L.meta(id)) << 22);
				else { const int i = (int)id - (int)LPE_RID; m = E ? sel3(i, rm1[0], rm1[1], rm1[2]) : sel3(i, rm0[0], rm0[1], rm0[2]); }
				const int c = cur[E];
				const uint32_t q0 = E ? tp1[0] : tp0[0], q1 = E ? tp1[1] : tp0[1];
				if ((c > 0 && q0 == pos) || (c > 1 && q1 == pos)) return;
				if (E) { PUT3(c, tm1[0], tm1[1], tm1[2], m); PUT3(c, tp1[0], tp1[1], tp1[2], pos); }
				else { PUT3(c, tm0[0], tm0[1], tm0[2], m); PUT3(c, tp0[0], tp0[1], tp0[2], pos); }
				if constexpr (SJ) {
					// a stored record keeps its junction record; one taken from this table gets the
					// junction search below (copy_vote_to_alignment_res runs after the position test,
					// core-junction.c:2413-2425)
					const int b = (E * 3 + c) * 4;
					uint32_t nib = 0;
					if (id >= LPE_RID) nib = (jm >> ((E * 3 + (int)id - (int)LPE_RID) * 4)) & 15u;
					else needj |= 1u << (E * 3 + c);
					tjm = (tjm & ~(15u << b)) | (nib << b);
				}
				cur[E] = c + 1;
			};
			if (ncomb > 0) {
				// merge_sort -> unstable selection sort ascending for <= 11 items (core.c:4716-4729)
				if (ncomb > 1) {
					int mj = 0;
					if (cs0 - cs1 > 0) mj = 1;
					if (ncomb > 2 && (mj ? cs1 : cs0) - cs2 > 0) mj = 2;
					if (mj == 1) { uint32_t a = ca0, b = cb0; int c = cs0; ca0 = ca1; cb0 = cb1; cs0 = cs1; ca1 = a; cb1 = b; cs1 = c; }
					else if (mj == 2) { uint32_t a = ca0, b = cb0; int c = cs0; ca0 = ca2; cb0 = cb2; cs0 = cs2; ca2 = a; cb2 = b; cs2 = c; }
					if (ncomb > 2 && cs1 - cs2 > 0) { uint32_t a = ca1, b = cb1; int c = cs1; ca1 = ca2; cb1 = cb2; cs1 = cs2; ca2 = a; cb2 = b; cs2 = c; }
				}
				// taken from the highest score down
#pragma unroll
				for (int e = 0; e < 2; e++)
#pragma unroll
					for (int i = 2; i >= 0; i--)
						if (i < ncomb && cur[e] < mb) emit(e, e ? sel3(i, cb0, cb1, cb2) : sel3(i, ca0, ca1, ca2));
			} else {
				// no pair: each end's simples with >= min_votes_first votes
#pragma unroll
				for (int e = 0; e < 2; e++)
					for (int i = 0; i < ns[e]; i++) {
						if (cur[e] >= mb) break;
						const uint32_t id = pl_get(pl[e], i);
						uint32_t pos;
						if (sv(e, id, pos) < mvf) continue;
						emit(e, id);
					}
			}
			if constexpr (SJ) {
				// junction part of copy_vote_to_alignment_res (core-junction.c:1073-1334) for every
				// record taken from this strand's tables, in lane_kernel's two phases; a minor half is
				// a slot of the same end's table.  List entries: end << 7 | record << 5 | slot.
				uint32_t *lst = L.jlist();
				int nl = 0;
				uint32_t ends_used = 0;
				for (int E = 0; E < 2 && !L.dfr; E++)
					for (int c = 0; c < cur[E] && !L.dfr; c++) {
						if (!((needj >> (E * 3 + c)) & 1u)) continue;
						const int sM = RM_SRC(E ? sel3(c, tm1[0], tm1[1], tm1[2]) : sel3(c, tm0[0], tm0[1], tm0[2])) & 63;
						const uint2 eM = L.slot(sM);
						const int vM = lm_votes(eM.y), stE = E ? step[1] : step[0];
						const int csM = (int)(*L.cw(st, sM, 0) & 0xffu), ceM = lcov_end(lm_last(eM.y), lm_x(eM.y), stE, lp.gap);
						for (uint32_t row = 0; row < LROWS && !L.dfr; row++) {
							uint32_t q = E ? L.template head<1>(row) : L.template head<0>(row);
							while (q != Lane<K, 2>::NIL) {
								const uint2 e2 = L.slot(q);
								const uint32_t qs = q;
								q = lm_next(e2.y);
								if ((int)qs == sM || vM < lm_votes(e2.y)) continue;
								const long long dist = (long long)eM.x - (long long)e2.x;
								if ((dist < 0 ? -dist : dist) > (long long)lp.max_intron) continue;
								const int cs2 = (int)(*L.cw(st, (int)qs, 0) & 0xffu), ce2 = lcov_end(lm_last(e2.y), lm_x(e2.y), stE, lp.gap);
								if (csM == cs2 || ceM == ce2) continue;
								if (csM > cs2 ? eM.x < e2.x : eM.x > e2.x) continue;   // test_junction_minor
								const int ov = csM > cs2 ? ce2 - csM : ceM - cs2;
								if (ov > 14 || abs((int)dist) < 6) continue;
								if (nl == LJLIST) { L.dfr = true; L.why = 2; break; }
								lst[nl * 64] = ((uint32_t)E << 8) | ((uint32_t)c << 6) | qs;
								nl++;
								ends_used |= 1u << E;
							}
						}
					}
				if (L.dfr) continue;
				if (ends_used & 1u) lcodes(lp.seq, lp.off, r, len[0], st ^ lp.rev, L.codes(0));
				if (ends_used & 2u) lcodes(lp.seq2, lp.off2, r, len[1], st ^ lp.rev2, L.codes(1));
				int Jk = -1, JE = 0, Jc = 0, Jv = 0, Jcs = 0, Jce = 0, Jsplit = 0, Jnormal = 0, Jf = -1;
				uint32_t Jpos = 0, Mpos = 0;
				int Mcs = 0, Mce = 0, sM = 0, stE = 0, rl = 0;
				auto flush = [&]() __attribute__((always_inline)) {
					if (Jf < 0) return;
					uint32_t *jw = L.jw(st, sM);
					jw[0] = (uint32_t)(uint16_t)Jsplit | ((uint32_t)(uint16_t)Jv << 16);
					jw[64] = ((uint32_t)(Jnormal ? 0 : 1) << 16) | ((uint32_t)(Jnormal ? 1 : 0) << 24);
					jw[128] = Jpos;
					jw[192] = (uint32_t)(uint16_t)Jcs | ((uint32_t)(uint16_t)Jce << 16);
					const int b = (JE * 3 + Jc) * 4;
					tjm = (tjm & ~(15u << b)) | ((1u | ((uint32_t)Jf << 1)) << b);
				};
				for (int k = 0; k < nl; k++) {
					const uint32_t ent = lst[k * 64];
					const int key = (int)(ent >> 6), qs = (int)(ent & 63u);
					if (key != Jk) {
						flush();
						Jk = key; JE = key >> 2; Jc = key & 3;
						Jv = 0; Jcs = 0; Jce = 0; Jsplit = 0; Jnormal = 0; Jf = -1; Jpos = 0;
						sM = RM_SRC(JE ? sel3(Jc, tm1[0], tm1[1], tm1[2]) : sel3(Jc, tm0[0], tm0[1], tm0[2])) & 63;
						stE = JE ? step[1] : step[0];
						rl = JE ? len[1] : len[0];
						const uint2 eM = L.slot(sM);
						Mpos = eM.x;
						Mcs = (int)(*L.cw(st, sM, 0) & 0xffu);
						Mce = lcov_end(lm_last(eM.y), lm_x(eM.y), stE, lp.gap);
					}
					const uint2 e2 = L.slot(qs);
					const int V = lm_votes(e2.y);
					const int cs2 = (int)(*L.cw(st, qs, 0) & 0xffu), ce2 = lcov_end(lm_last(e2.y), lm_x(e2.y), stE, lp.gap);
					// is_better_inner (core-junction.c:961)
					const int oldi = (int)labs32u(Mpos - Jpos), intr = (int)labs32u(Mpos - e2.x);
					const int cl = ce2 - cs2, jl = Jce - Jcs;
					if (!(V > Jv || (V == Jv && cl > jl) || (V == Jv && cl == jl && intr < oldi))) continue;
					const int gs = Mcs > cs2 ? ce2 - 8 : Mce - 8;
					const int ge = Mcs < cs2 ? cs2 + 8 : Mcs + 8;
					const int normal = 1 != (int)(Mcs > cs2) + (int)(Mpos > e2.x);
					int split = 0, gtag = 0;
					const int best = ldonor(lp, L.codes(JE), rl, Mpos < e2.x ? Mpos : e2.x, Mpos > e2.x ? Mpos : e2.x, normal,
					                        gs > 0 ? gs : 0, ge < rl ? ge : rl, split, gtag);
					if (best > 0) {
						Jpos = e2.x; Jv = V; Jcs = cs2; Jce = ce2; Jsplit = split; Jnormal = normal;
						Jf = best < 290000 ? 3 : (gtag ? 1 : 0);
					}
				}
				flush();
			}
#pragma unroll
			for (int i = 0; i < 3; i++) {
				if (i < cur[0]) {
					rm0[i] = tm0[i]; rp0[i] = tp0[i];
					if (SJ) jm = (jm & ~(15u << (i * 4))) | (tjm & (15u << (i * 4)));
				} else rm0[i] = RM_SETV(rm0[i], 0);
				if (i < cur[1]) {
					rm1[i] = tm1[i]; rp1[i] = tp1[i];
					if (SJ) jm = (jm & ~(15u << ((3 + i) * 4))) | (tjm & (15u << ((3 + i) * 4)));
				} else rm1[i] = RM_SETV(rm1[i], 0);
			}
		}
		if (!L.dfr) ncand += (unsigned long long)nc_read;
		// ---- the pair's 2 x multi_best records
		if (!L.dfr) {
#pragma unroll
			for (int e = 0; e < 2; e++) {
				uint32_t *dst = (uint32_t *)(lp.out + ((size_t)r * 2 + e) * mb * 68);
				for (int i = 0; i < mb; i++) {
					const uint32_t m = e ? sel3(i, rm1[0], rm1[1], rm1[2]) : sel3(i, rm0[0], rm0[1], rm0[2]);
					const uint32_t pos = e ? sel3(i, rp1[0], rp1[1], rp1[2]) : sel3(i, rp0[0], rp0[1], rp0[2]);
					uint32_t w[17];
					write_record(L, RM_SRC(m), pos, RM_V(m), RM_U(m), RM_EXT(m), step[e], lp.gap, w);
					if constexpr (SJ) {
						// the record's subjunc_result_t (empty without a minor half; a zero-vote record
						// keeps the stale one with minor_votes 0)
						const uint32_t nib = (jm >> ((e * 3 + i) * 4)) & 15u;
						uint4 jr = make_uint4(0u, 0u, 0u, 0u);
						const int src = RM_SRC(m);
						if (src >= 0 && (nib & 1u)) {
							const uint32_t *jw = L.jw(src >> 6, src & 63);
							jr = make_uint4(RM_V(m) > 0 ? jw[0] : (jw[0] & 0xffffu), jw[64], jw[128], jw[192]);
							w[1] |= (nib >> 1) & 3u;
						}
						*(uint4 *)(lp.jout + (((size_t)r * 2 + e) * mb + i) * 16) = jr;
					}
#pragma unroll
					for (int k = 0; k < 17; k++) dst[i * 17 + k] = w[k];
					nres += RM_V(m) > 0;
				}
				if constexpr (SJ) {
					if (lp.bm_out) {
						uint16_t *bd = lp.bm_out + ((size_t)r * 2 + e) * SVG_BIG_MARGIN_WORDS;
#pragma unroll
						for (int k = 0; k < 3; k++) {
							bd[3 * k] = (uint16_t)bv[e][k];
							bd[3 * k + 1] = (uint16_t)(bs[e][k] & 0xffffu);
							bd[3 * k + 2] = (uint16_t)(bs[e][k] >> 16);
						}
					}
				}
			}
		}
		const unsigned long long dm = __ballot(L.dfr && live);
		if (dm) {
			uint32_t base = 0;
			const int leader = __ffsll((long long)dm) - 1;
			if (L.lane == leader) base = atomicAdd(lp.defer_count, (uint32_t)__popcll(dm));
			base = __shfl(base, leader);
			if (L.dfr && live) lp.defer_list[base + __popcll(dm & ((1ull << L.lane) - 1ull))] = r;
			ndef += (unsigned long long)__popcll(dm);
		}
		if (lp.stats) {
			nwhy1 += (unsigned long long)__popcll(__ballot(L.dfr && live && L.why == 1));
			nwhy2 += (unsigned long long)__popcll(__ballot(L.dfr && live && L.why == 2));
			nwhy3 += (unsigned long long)__popcll(__ballot(L.dfr && live && L.why == 3));
		}
	}
	if (lp.stats) {
		for (int o = 32; o; o >>= 1) { nres += __shfl_xor(nres, o); ncand += __shfl_xor(ncand, o); }
		if (L.lane == 0) {
			atomicAdd(&lp.stats[3], nres);
			if (lp.final_pass) atomicAdd(&lp.stats[4], ndef);
			unsigned long long *d = lp.stats + lp.stat_base;
			atomicAdd(&d[0], nwhy1);
			atomicAdd(&d[1], nwhy2);
			atomicAdd(&d[2], nwhy3);
			atomicAdd(&d[3], ncand);
			atomicAdd(&d[4], ndef);
		}
	}
}

// ---------------------------------------------------------------------------------------------
// count bins (fused SE path): thread per read, the same eligibility tests and per-strand
// candidate counts the lane kernel starts with (its probe records, SoA); reads past the lane
// limits go straight to the deferral list, the rest to bin lbin_of(larger strand count)
// ---------------------------------------------------------------------------------------------
// Block tiles of LBT consecutive reads: the tile's lists are built in LDS (local offsets), then
// one global atomic per list and tile reserves the output range (per-wave global atomics on five
// counters serialised the kernel), and each list goes out in the tile's read order.
#define LBT 1024   // 4 rounds of 256 reads per tile, ~4 tiles per CU at 1M reads (latency hidden across blocks)
template <int NPF>
__global__ void __launch_bounds__(256) lane_bin_kernel(LParams lp)
{
	__shared__ uint16_t lst[LBINS + 1][LBT];   // list LBINS: deferred
	__shared__ uint32_t lcnt[LBINS + 1], gbase[LBINS + 1];
	const int lane = (int)__lane_id(), tid = (int)threadIdx.x;
	unsigned long long ndef = 0;
	for (uint32_t t0 = blockIdx.x * LBT; t0 < lp.n; t0 += gridDim.x * LBT) {
		if (tid <= LBINS) lcnt[tid] = 0;
		__syncthreads();
		for (int i = 0; i < LBT / 256; i++) {
			const uint32_t loc = (uint32_t)(i * 256 + tid), r = t0 + loc;
			const bool live = r < lp.n;
			int len = live ? lp.len[r] : 0;
			if (len > SVG_READ_KEEP) len = SVG_READ_KEEP;
			bool dfr = lp.defer_all != 0;
			int applied = 0;
			if (len >= 15 + lp.gap) {
				const int cr = (len - 15 - lp.gap) << 16;
				int step = cr / (lp.total_subreads - 1);
				if (step < (lp.gap << 16)) step = lp.gap << 16;
				applied = 1 + cr / step;
			}
			if (len < 15 + lp.gap || len > 160 || applied > 31 || applied * lp.gap > NPF || applied * lp.gap > lp.nps) dfr = true;
			const int np = applied * lp.gap;
			int mx = 0;
#pragma unroll
			for (int st = 0; st < 2; st++) {
				int cnt = 0;
#pragma unroll
				for (int p = 0; p < NPF; p++) {
					const uint32_t y = live && !dfr && p < np ? lp.precs[(size_t)(st * lp.nps + p) * lp.n + r].y : 0u;
					cnt += (int)((y & 0xffffu) + (y >> 16));
				}
				mx = cnt > mx ? cnt : mx;
			}
			if (mx > lp.cap) dfr = true;
			const int cl = dfr ? LBINS : lbin_of(mx);
#pragma unroll
			for (int q = 0; q <= LBINS; q++) {
				const unsigned long long bm = __ballot(live && cl == q);
				if (!bm) continue;
				const int leader = __ffsll((long long)bm) - 1;
				uint32_t base = 0;
				if (lane == leader) base = atomicAdd(&lcnt[q], (uint32_t)__popcll(bm));
				base = __shfl(base, leader);
				if (live && cl == q) lst[q][base + __popcll(bm & ((1ull << lane) - 1ull))] = (uint16_t)loc;
			}
		}
		__syncthreads();
		if (tid <= LBINS) {
			const uint32_t c = lcnt[tid];
			gbase[tid] = c ? atomicAdd(tid == LBINS ? lp.defer_count : &lp.bin_count[tid], c) : 0u;
		}
		__syncthreads();
#pragma unroll
		for (int q = 0; q <= LBINS; q++) {
			const uint32_t c = lcnt[q];
			uint32_t *dst = (q == LBINS ? lp.defer_list : lp.bins + (size_t)q * lp.n) + gbase[q];
			for (uint32_t j = (uint32_t)tid; j < c; j += 256u) dst[j] = t0 + lst[q][j];
		}
		ndef += lcnt[LBINS];
		__syncthreads();   // lcnt / lst are reused by the next tile
	}
	if (lp.stats && tid == 0 && ndef) {
		if (lp.final_pass) atomicAdd(&lp.stats[4], ndef);
		atomicAdd(&lp.stats[lp.stat_base + 0], ndef);   // reason 1: candidates > CAP or length
		atomicAdd(&lp.stats[lp.stat_base + 4], ndef);
	}
}

// ---------------------------------------------------------------------------------------------
// host: two lane passes for one chunk (SE align), then the wave kernel for what is left
//   pass 1 (light): every read, <= 40 candidates and <= 20 vote-table slots per strand
//   pass 2 (heavy, SVG_LANE=3 only): the reads pass 1 deferred (up to n/4 of them), <= 192
//                   candidates and <= 64 slots per strand.  Measured at C3 it costs more than
//                   it saves (64-slot tables: 5 waves/CU, long row walks, and most repeat-family
//                   reads still overflow), so the wave kernel takes pass 1's deferrals directly.
// ---------------------------------------------------------------------------------------------
#ifndef LANE_K1
// slots per lane: 16 = 8 KB LDS per wave.  20 (10 KB) filled the 4 waves/SIMD the VGPRs allow, but
// beside the wave kernel of the previous chunk (~89 KB of a CU's LDS) the lane kernel then fits 7
// waves per CU instead of 8: 16 measured faster at C3 in one process, 99.8 vs 101.8 ms/step with
// either build first (profiles/r04/z/ab_k20_vs_k16.txt, r04/y/), though 3% more reads need the
// wave kernel (5.94M vs 5.77M per 50M)
#define LANE_K1 16
#endif
// subjunc and the unfused (gather kernel) path keep 20: a deferred subjunc read costs the wave
// kernel far more (C5 with 16: 148.4 vs 164.8 Mreads/s, profiles/r04/aa/bench_c5.json)
#ifndef LANE_K1_WIDE
#define LANE_K1_WIDE 20
#endif
#define LANE_NPF 10   // probe records per strand held in registers by the fused light pass
#define LANE_NPF_SJ 14   // subjunc: -n 14
#define LANE_CAP1 40

template <int K, int NPF>
static int lane_launch(svg_index *h, LParams &lp, uint32_t **cold, size_t *cold_words, hipStream_t st)
{
	const size_t lds = (size_t)K * 64 * sizeof(uint2);
	int per_cu = (int)(160 * 1024 / lds);
	if (per_cu > 32) per_cu = 32;
	uint64_t blocks = (uint64_t)h->n_cu * per_cu, need_b = (lp.n + 63) / 64;
	if (blocks > need_b) blocks = need_b;
	if (blocks < 1) blocks = 1;
	const size_t words = blocks * (size_t)(lane_cold_words(K, lp.jout != NULL) * 64);
	if (words > *cold_words) {
		hipFree(*cold);
		*cold = NULL;
		*cold_words = 0;
		if (dmalloc(h, (void **)cold, words * 4 + 256)) return SVG_E_NOMEM;
		*cold_words = words;
	}
	lp.cold = *cold;
	int rc = svg_timing_mark(h, 3, 0, st);
	if (rc) return rc;
	if (lp.jout) hipLaunchKernelGGL((lane_kernel<K, NPF == 0 ? 0 : LANE_NPF_SJ, true>), dim3((unsigned)blocks), dim3(64), lds, st, lp);
	else hipLaunchKernelGGL((lane_kernel<K, NPF, false>), dim3((unsigned)blocks), dim3(64), lds, st, lp);
	HIPCHK(hipGetLastError());
	return svg_timing_mark(h, 3, 1, st);
}

static int gather_launch(svg_index *h, const GParams &g, hipStream_t st)
{
	uint64_t blocks = ((uint64_t)2 * g.cs + 255) / 256, bmax = (uint64_t)h->n_cu * 32;
	if (blocks > bmax) blocks = bmax;
	if (blocks < 1) blocks = 1;
	int rc = svg_timing_mark(h, 2, 0, st);
	if (rc) return rc;
	hipLaunchKernelGGL(gather_kernel, dim3((unsigned)blocks), dim3(256), 0, st, g);
	HIPCHK(hipGetLastError());
	return svg_timing_mark(h, 2, 1, st);
}

int svg_lane_eligible(const svg_index *h, const svg_params *p, int paired, int sj)
{
	if (svg_get_option("lane") == 3) return 0;   // wave kernel only (testing)
	if (h->max_read_len > 160) return 0;
	// subjunc: junction search on (the lane paths carry big-margin records and defer every read
	// or pair that needs donor scoring)
	if (sj && (!p->do_breakpoint_detection || p->max_insertion_at_junctions)) return 0;
	int tol = p->max_indel_length < 16 ? p->max_indel_length : 16;
	if (tol > 5 || p->total_subreads > 31 || p->multi_best > 3 || p->top_scores != 3) return 0;
	if (!paired && p->max_vote_simples > 3) return 0;
	if (paired && p->max_vote_combinations > 3) return 0;
	return 1;
}


#define LANE_PE_CAP 40

// paired-end: lane_pe_kernel over every pair of the chunk; deferred pairs listed for vote_kernel
int svg_lane_pe_chunk(svg_index *h, int slot, const svg_params *p, const uint16_t *len1, const uint16_t *len2, uint32_t n,
                      const uint2 *precs, int nps, uint8_t *out, uint8_t *jout, uint16_t *bm_out, const char *seq1,
                      const uint64_t *off1, const char *seq2, const uint64_t *off2, unsigned long long *stats,
                      uint32_t **defer_list, uint32_t **defer_count, hipStream_t st)
{
	if (slot < 0 || slot > 2) { svg_set_error("chunk slot %d out of range", slot); return SVG_E_ARG; }   // [3]-slot buffers
	const size_t o_l1 = 0, o_cnt = (o_l1 + (size_t)4 * n + 255) & ~(size_t)255, need = o_cnt + 256;
	if (need > h->lane_cap[slot]) {
		hipFree(h->d_lane[slot]);
		h->d_lane[slot] = NULL;
		h->lane_cap[slot] = 0;
		if (dmalloc(h, &h->d_lane[slot], need)) return SVG_E_NOMEM;
		h->lane_cap[slot] = need;
	}
	uint8_t *b = (uint8_t *)h->d_lane[slot];
	uint32_t *cnt = (uint32_t *)(b + o_cnt);   // [0] deferrals, [2] wave-kernel work counter
	HIPCHK(hipMemsetAsync(cnt, 0, 16, st));
	if (nps > (jout ? LANE_NPF_SJ : LANE_NPF)) { svg_set_error("lane_pe: %d probes per strand", nps); return SVG_E_UNSUPPORTED; }
	LParams lp;
	memset(&lp, 0, sizeof lp);
	lp.len = len1; lp.len2 = len2; lp.n = n; lp.cap = LANE_PE_CAP;
	lp.precs = precs; lp.vals = h->dix.vals; lp.nps = nps;
	lp.gap = h->dix.gap; lp.total_subreads = p->total_subreads;
	lp.tol = p->max_indel_length < 16 ? p->max_indel_length : 16;
	lp.low = h->dix.start_base_offset;
	lp.high = h->dix.start_base_offset + h->dix.length;
	lp.multi_best = p->multi_best; lp.max_vote_simples = p->max_vote_simples; lp.cutoff = p->max_vote_number_cutoff;
	lp.min_votes_first = p->min_votes_first; lp.min_votes_second = p->min_votes_second;
	lp.chr_end = h->dix.chr_end; lp.n_chr = (int)h->dix.n_chr; lp.padding = h->dix.padding;
	lp.min_pair = p->min_pair_distance; lp.max_pair = p->max_pair_distance; lp.mvc = p->max_vote_combinations;
	// 96 -> 256: C5pe deferrals 34% -> 21% of the pairs, 942 -> 779 ms/step (profiles/r03/sweeps/c5pe_pairs_*.json)
	lp.max_pairs = 256;   // measured: 96 -> 256 pairs cut C5pe deferrals 8.57M -> 5.18M of 25M; 1024 the same
	lp.out = out;
	lp.jout = jout;
	lp.bm_out = jout ? bm_out : NULL;
	lp.bm_size = p->do_big_margin_filtering_for_junctions ? p->big_margin_record_size : 0;
	lp.max_intron = p->maximum_intron_length;
	// donor scoring (subjunc): both ends' read text and the .array
	lp.seq = seq1; lp.off = off1; lp.seq2 = seq2; lp.off2 = off2;
	lp.values = h->dix.values;
	lp.v_sbo = h->dix.start_base_offset; lp.v_len = h->dix.length; lp.v_start = h->dix.start_point;
	lp.v_bytes = h->dix.values_bytes;
	lp.need_donor = p->check_donor_at_junctions != 0;
	lp.prefer_donor = p->prefer_donor_receptor_junctions != 0;
	lp.allow_mm = p->more_accurate_fusions ? 0 : 1;
	lp.rev = p->reverse_r1 != 0;
	lp.rev2 = p->reverse_r2 != 0;
	lp.defer_list = (uint32_t *)(b + o_l1);
	lp.defer_count = cnt;
	lp.defer_all = svg_get_option("lane") == 2;
	lp.stats = stats;
	lp.stat_base = 16;
	lp.final_pass = 1;
	lp.cs = n;
	constexpr int K = LANE_PE_K;
	const size_t lds = (size_t)K * 64 * sizeof(uint2);
	int per_cu = (int)(160 * 1024 / lds);
	if (per_cu > 32) per_cu = 32;
	uint64_t blocks = (uint64_t)h->n_cu * per_cu, need_b = (n + 63) / 64;
	if (blocks > need_b) blocks = need_b;
	if (blocks < 1) blocks = 1;
	const size_t words = blocks * (size_t)(lane_cold_words(K, jout != NULL, 2) * 64);
	if (words > h->lscratch_words) {
		hipFree(h->d_lscratch);
		h->d_lscratch = NULL;
		h->lscratch_words = 0;
		if (dmalloc(h, (void **)&h->d_lscratch, words * 4 + 256)) return SVG_E_NOMEM;
		h->lscratch_words = words;
	}
	lp.cold = h->d_lscratch;
	int rc = svg_timing_mark(h, 3, 0, st);
	if (rc) return rc;
	if (jout) hipLaunchKernelGGL((lane_pe_kernel<K, LANE_NPF_SJ, true>), dim3((unsigned)blocks), dim3(64), lds, st, lp);
	else hipLaunchKernelGGL((lane_pe_kernel<K, LANE_NPF, false>), dim3((unsigned)blocks), dim3(64), lds, st, lp);
	HIPCHK(hipGetLastError());
	if ((rc = svg_timing_mark(h, 3, 1, st))) return rc;
	*defer_list = lp.defer_list;
	*defer_count = cnt;
	return 0;
}

int svg_lane_chunk(svg_index *h, int slot, const svg_params *p, const uint16_t *len, uint32_t n, const uint2 *precs, int nps,
                   uint8_t *out, uint8_t *jout, uint16_t *bm, const char *seq, const uint64_t *off,
                   unsigned long long *stats, uint32_t **defer_list, uint32_t **defer_count, hipStream_t st)
{
	if (slot < 0 || slot > 2) { svg_set_error("chunk slot %d out of range", slot); return SVG_E_ARG; }   // [3]-slot buffers
	// buffers: cand/cpk/cnt over n columns (unfused gather), deferral list, counters, count bins
	const size_t o_c1 = 0, o_p1 = o_c1 + (size_t)8 * LANE_CAP1 * n, o_n1 = o_p1 + (size_t)4 * LANE_CAP1 * n;
	const size_t o_l1 = (o_n1 + (size_t)4 * n + 255) & ~(size_t)255;
	const size_t o_cnt = o_l1 + (size_t)4 * n + 256, o_bin = o_cnt + 256, need = o_bin + (size_t)4 * LBINS * n + 256;
	if (need > h->lane_cap[slot]) {
		hipFree(h->d_lane[slot]);
		h->d_lane[slot] = NULL;
		h->lane_cap[slot] = 0;
		if (dmalloc(h, &h->d_lane[slot], need)) return SVG_E_NOMEM;
		h->lane_cap[slot] = need;
	}
	uint8_t *b = (uint8_t *)h->d_lane[slot];
	// [0] deferrals, [2] wave-kernel work counter, [4..7] count-bin sizes
	uint32_t *cnt = (uint32_t *)(b + o_cnt);
	HIPCHK(hipMemsetAsync(cnt, 0, 32, st));
	GParams g;
	g.precs = precs; g.len = len; g.vals = h->dix.vals; g.n = n; g.nps = nps; g.gap = h->dix.gap;
	g.total_subreads = p->total_subreads; g.cap = LANE_CAP1;
	g.cand = (uint32_t *)(b + o_c1); g.cpk = (uint16_t *)(b + o_p1); g.ccnt = (uint16_t *)(b + o_n1);
	g.cs = n; g.idx = NULL; g.idx_count = NULL;
	// reads of <= LANE_NPF probes per strand (the full index at the default -n): the gather is
	// fused into the lane kernel; otherwise the gather kernel writes candidate lists first
	const bool sjm = jout != NULL;   // subjunc (lane_kernel<..., true>)
	const bool fused = nps <= (sjm ? LANE_NPF_SJ : LANE_NPF) && !svg_get_option("lane_unfused");
	int rc = 0;
	if (!fused && (rc = gather_launch(h, g, st))) return rc;
	LParams lp;
	lp.cand = g.cand; lp.cpk = g.cpk; lp.ccnt = g.ccnt; lp.len = len; lp.n = n; lp.cap = LANE_CAP1;
	lp.precs = precs; lp.vals = h->dix.vals; lp.nps = nps;
	lp.gap = h->dix.gap; lp.total_subreads = p->total_subreads;
	lp.tol = p->max_indel_length < 16 ? p->max_indel_length : 16;
	lp.low = h->dix.start_base_offset;
	lp.high = h->dix.start_base_offset + h->dix.length;
	lp.multi_best = p->multi_best; lp.max_vote_simples = p->max_vote_simples; lp.cutoff = p->max_vote_number_cutoff;
	lp.min_votes_first = p->min_votes_first; lp.min_votes_second = p->min_votes_second;
	lp.out = out;
	lp.jout = jout;
	lp.bm_out = p->do_big_margin_filtering_for_junctions ? bm : NULL;
	lp.bm_size = p->do_big_margin_filtering_for_junctions ? p->big_margin_record_size : 0;
	lp.max_intron = p->maximum_intron_length;
	// donor scoring (subjunc): the chunk's read text and the .array
	lp.seq = seq; lp.off = off;
	lp.values = h->dix.values;
	lp.v_sbo = h->dix.start_base_offset; lp.v_len = h->dix.length; lp.v_start = h->dix.start_point;
	lp.v_bytes = h->dix.values_bytes;
	lp.need_donor = p->check_donor_at_junctions != 0;
	lp.prefer_donor = p->prefer_donor_receptor_junctions != 0;
	lp.allow_mm = p->more_accurate_fusions ? 0 : 1;
	lp.rev = p->reverse_r1 != 0;
	lp.defer_list = (uint32_t *)(b + o_l1);
	lp.defer_count = cnt;
	lp.defer_all = svg_get_option("lane") == 2;
	lp.stats = stats;
	lp.stat_base = 16;
	lp.final_pass = 1;
	lp.cs = n; lp.idx = NULL; lp.idx_count = NULL;
	lp.bins = NULL; lp.bin_count = NULL;
	{
		// option lane_cap: candidates per strand (<= 64 fused); lane_bin 2: no count bins
		const int oc = (int)svg_get_option("lane_cap");
		if (oc > 0 && oc <= LANE_CAP1) lp.cap = oc;
		if (oc > LANE_CAP1 && fused) lp.cap = oc < 64 ? oc : 64;
		// count bins for the fused single-pass path: one thread per read sorts the chunk's reads into
		// LBINS lists by candidate count (and defers the over-cap ones) before the lane kernel
		if (fused) {
			lp.bins = (uint32_t *)(b + o_bin);
			lp.bin_count = cnt + 4;
			uint64_t bb = ((uint64_t)n + LBT - 1) / LBT, bmax = (uint64_t)h->n_cu * 8;
			if (bb > bmax) bb = bmax;
			if (bb < 1) bb = 1;
			if (sjm) hipLaunchKernelGGL(lane_bin_kernel<LANE_NPF_SJ>, dim3((unsigned)bb), dim3(256), 0, st, lp);
			else hipLaunchKernelGGL(lane_bin_kernel<LANE_NPF>, dim3((unsigned)bb), dim3(256), 0, st, lp);
			HIPCHK(hipGetLastError());
		}
		if (!fused) rc = lane_launch<LANE_K1_WIDE, 0>(h, lp, &h->d_lscratch, &h->lscratch_words, st);
		else if (sjm) rc = lane_launch<LANE_K1_WIDE, LANE_NPF_SJ>(h, lp, &h->d_lscratch, &h->lscratch_words, st);
		else rc = lane_launch<LANE_K1, LANE_NPF>(h, lp, &h->d_lscratch, &h->lscratch_words, st);
	}
	if (rc) return rc;
	*defer_list = lp.defer_list;
	*defer_count = cnt;
	return 0;
}
