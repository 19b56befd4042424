// svg_fragile.hip -- fragile junction voting of subjunc reads longer than 160 bases
// (core_fragile_junction_voting, core-junction.c:5151-5422; do_voting calls it per index block,
// strand and read end, core.c:3138-3142) on the GPU: one wavefront per ~60-base window.
//
//   stage    the window of the strand's text (strand 1 = reverse_read of the fetched read) in LDS
//   probe    lane = subread probe: offsets every 3.00001 bases (x gap slots), genekey2int, and
//            gehash_go_q's search (sorted-hashtable.c:750-811): binary search on the bucket's
//            int16 keys, back to the first equal key, the run length
//   vote     candidates in go_q's order (probe, then the run from its first item), each voted
//            into a 30 x 24 LDS table with the go_X round-0 state machine (tolerance 5; lanes =
//            the slots of rows kv/5, +5, -5 in scan order, a ballot finds the first taker)
//   decide   lane = slot: the top-vote slots with a second recorder section (reported), the
//            last top-vote slot (select_best_vote, sorted-hashtable.c:1128), the best second
//            half (core_select_best_matching_halves_maxone, core-junction.c:4741-4896) by a
//            64-bit max over (score, row-major index); lane = split point: core13_test_donor
//            (core-junction.c:5027-5141) by a max over (score, -split)
// The host turns the windows into events (svg_events_add_batch2, svg_events.c).
// Integer work only: no MFMA.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "subread_vote.h"
#include "svg_internal.h"
#include "svg_device.h"

#define F_ROWS 30
#define F_SPACE 24
#define F_SLOTS (F_ROWS * F_SPACE)
#define F_REC 21          // MAX_INDEL_SECTIONS * 3
#define F_WIN 60          // EXON_LARGE_WINDOW
#define F_TOL 5
#define F_MAXW 96         // longest window (the last one: rl - cursor, ~60)
#define F_MAXP 64         // probes per window (15 subreads x 3 gap slots at 60 bases)
#define F_STEPS 72        // (int)(3.00001f * k), k < F_STEPS

struct FJob {             // one window, in the result's order
	uint64_t text;        // first base of the read's fetched (strand-0) text in the upload
	uint32_t read;
	uint16_t rl, cursor, wl;
	uint8_t strand, end, window, pad;
};

struct FParams {
	DevIndex ix;
	const char *text;
	const FJob *jobs;
	uint32_t n_jobs;
	int block;
	const int16_t *f3;    // (int)(3.00001f * k): the reference's float subread stepping
	uint32_t low, high;   // start_base_offset, start_base_offset + length of the block's array
	svg_fragile_window *wout;
	svg_fragile_slot *sout;
	uint32_t *scount;     // slots written (may exceed scap: the host retries with room)
	uint32_t scap;
	int literal;          // option keys_literal: the literal bucket search for every probe (A/B, tests)
};

struct FLDS {
	uint32_t pos[F_SLOTS];
	uint32_t meta[F_SLOTS];          // votes | last << 8 | toli << 16 | (u8)cursor << 24
	uint16_t cov[F_SLOTS];           // coverage_start | coverage_end << 8 (window <= 96 bases)
	int8_t rec[F_SLOTS][F_REC + 3];  // indel recorder (values fit int8: subread numbers <= 32, |d| <= 5)
	char text[F_MAXW + 32];
	uint32_t pfirst[F_MAXP], pcnt[F_MAXP], pcum[F_MAXP + 1];
	uint16_t ppk[F_MAXP];            // kP1 | off << 6
};

__device__ __forceinline__ int f_lane() { return __lane_id(); }
__device__ __forceinline__ void f_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); }
__device__ __forceinline__ int f_rd(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint32_t f_row(uint32_t x) { return (x / 5u) % F_ROWS; }
__device__ __forceinline__ char f_comp(char c)
{
	return c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : (c == 'T' || c == 'U') ? 'A' : 'N';
}
__device__ __forceinline__ uint32_t f_b2i(char c) { return c < 'G' ? (c == 'A' ? 0u : 2u) : (c == 'G' ? 1u : 3u); }

// gvindex_get, gene-value-index.c:96-107
__device__ __forceinline__ char f_gv(const DevIndex &x, uint32_t pos)
{
	const uint32_t byte = (pos - x.start_base_offset) >> 2;
	if (byte >= x.values_bytes - 1) return 'N';
	const int b = (x.values[byte] >> ((pos & 3u) * 2u)) & 3;
	return b == 0 ? 'A' : b == 1 ? 'G' : b == 2 ? 'C' : 'T';
}
__device__ __forceinline__ char f_cpl(char c) { return c == 'A' ? 'T' : c == 'T' ? 'A' : c == 'G' ? 'C' : c == 'C' ? 'G' : c; }

// match_chro, gene-value-index.c:856-959 (base space), either strand
__device__ int f_match(const DevIndex &x, const char *read, uint32_t pos, int len, int neg)
{
	if ((uint32_t)(pos + (uint32_t)len) >= x.length + x.start_point) return 0;
	if (pos > 0xffff0000u) return 0;
	int ret = 0;
	if (neg) {
		for (int i = len - 1; i >= 0; i--) {
			const char t = f_gv(x, pos + (uint32_t)(len - 1 - i));
			const char r = read[i];
			ret += (t == 'A' && r == 'T') || (t == 'T' && r == 'A') || (t == 'G' && r == 'C') || (t == 'C' && r == 'G');
		}
		return ret;
	}
	uint32_t byte = (pos - x.start_base_offset) >> 2, bit = (pos & 3u) * 2u;
	if (byte >= x.values_bytes) return 0;
	int iv = (int)(int8_t)x.values[byte];
	for (int i = 0; i < len; i++) {
		const int tt = (iv >> bit) & 3;
		const char r = read[i];
		ret += r == 'A' ? tt == 0 : r == 'G' ? tt == 1 : r == 'C' ? tt == 2 : r == 0 ? 0 : tt == 3;
		bit += 2;
		if (bit == 8) {
			byte++;
			if (byte == x.values_bytes) return 0;
			iv = (int)(int8_t)x.values[byte];
			bit = 0;
		}
	}
	return ret;
}

// gvindex_get_string(h, x, pos, 2, neg), gene-value-index.c:1118-1136
__device__ __forceinline__ void f_2base(const DevIndex &x, uint32_t pos, int neg, char &h0, char &h1)
{
	if (!neg) { h0 = f_gv(x, pos); h1 = f_gv(x, pos + 1); }
	else { h1 = f_cpl(f_gv(x, pos)); h0 = f_cpl(f_gv(x, pos + 1)); }
}
__device__ __forceinline__ bool f_eq(char a0, char a1, char t0, char t1) { return a0 == t0 && a1 == t1; }
__device__ __forceinline__ bool f_donor_part(char a, char b)
{
	return f_eq(a, b, 'G', 'T') || f_eq(a, b, 'A', 'G') || f_eq(a, b, 'A', 'C') || f_eq(a, b, 'C', 'T');
}
// paired_chars_part, core-junction.c:4366-4374
__device__ __forceinline__ bool f_paired(char a0, char a1, char b0, char b1, int rev)
{
	const bool c2 = (f_eq(a0, a1, 'G', 'T') && f_eq(b0, b1, 'A', 'G')) || (f_eq(a0, a1, 'A', 'G') && f_eq(b0, b1, 'G', 'T')) ||
	                (f_eq(a0, a1, 'C', 'T') && f_eq(b0, b1, 'A', 'C')) || (f_eq(a0, a1, 'A', 'C') && f_eq(b0, b1, 'C', 'T'));
	if (!c2) return false;
	if (rev) return f_eq(a0, a1, 'A', 'G') || f_eq(a0, a1, 'A', 'C');
	return f_eq(a0, a1, 'C', 'T') || f_eq(a0, a1, 'G', 'T');
}

// locate_gene_position_max(..., NULL, NULL, rl = 0), gene-algorithms.c:441-511: the contig
// index, -1 for the reference's NULL name
__device__ int f_locate(const DevIndex &x, uint32_t linear)
{
	int lo = 0, hi = (int)x.n_chr, n;
	for (;;) {
		if (hi <= lo + 1) { n = lo - 2 > 0 ? lo - 2 : 0; break; }
		const int mid = (lo + hi) / 2;
		if (x.chr_end[mid] > linear) hi = mid; else lo = mid + 1;
	}
	for (; n < (int)x.n_chr; n++) {
		const uint32_t c = x.chr_end[n];
		if (c > linear) {
			const int pos = n == 0 ? (int)linear : (int)(linear - x.chr_end[n - 1]);
			if (linear > c + 15u - (uint32_t)x.padding) return -1;
			if (pos < x.padding) return -1;
			return n;
		}
	}
	return -1;
}

// the go_X round-0 tally (sorted-hashtable.c:1015-1106 as gehash_go_q runs it, 815-927) for one
// candidate: returns nothing; the table lives in L, items[] (row occupancy) in lanes 0..29 of
// `items`, max_vote in `maxv`
__device__ void f_vote(FLDS *L, int &items, int &maxv, uint32_t kv, int kP1, int off, uint32_t low, uint32_t high_w)
{
	const int lane = f_lane();
	const uint32_t r0 = f_row(kv), rp = f_row(kv + 5u), rm = f_row(kv - 5u);
	const int n0 = __shfl(items, (int)r0), np_ = __shfl(items, (int)rp), nm = __shfl(items, (int)rm);
	bool done = false;
	// scan order: row r0 slots, row rp slots, row rm slots; lane = position (two passes for > 64)
	for (int base = 0; base < n0 + np_ + nm && !done; base += 64) {
		const int q = base + lane;
		const bool valid = q < n0 + np_ + nm;
		const uint32_t row = q < n0 ? r0 : (q < n0 + np_ ? rp : rm);
		const int sl = q < n0 ? q : (q < n0 + np_ ? q - n0 : q - n0 - np_);
		const int slot = valid ? (int)row * F_SPACE + sl : 0;
		const uint32_t P = L->pos[slot], M = L->meta[slot];
		const int d = (int)(kv - P);
		const bool match = valid && d >= -F_TOL && d <= F_TOL;
		if (!__ballot(match)) continue;
		int votes = (int)(M & 0xffu), last = (int)((M >> 8) & 0xffu), tl = (int)((M >> 16) & 0xffu), cur = (int)(int8_t)(M >> 24);
		bool rb = false;
		if (match && kP1 == last && tl > 0) {   // roll-back (sorted-hashtable.c:849-862)
			int md = tl >= 3 ? (int)L->rec[slot][tl - 1] : 0;
			const int nd = md - d;
			md -= (int)L->rec[slot][tl + 2];
			rb = abs(md) > abs(nd);
		}
		const int last2 = rb ? last - 1 : last;
		const unsigned long long wm = __ballot(match && kP1 > last2);
		const int wl = wm ? __ffsll((long long)wm) - 1 : 64;
		if (match && lane <= wl) {
			if (rb) { tl -= 3; last -= 1; votes -= 1; }
			if (lane == wl) {
				votes += 1;
				const int ce = (int)(L->cov[slot] >> 8);
				if (off + 16 > ce) L->cov[slot] = (uint16_t)((L->cov[slot] & 0xffu) | ((uint32_t)(off + 16) << 8));
				if (d == cur) L->rec[slot][tl + 1] = (int8_t)kP1;
				else {
					const int t2 = tl + 3;
					if (t2 < F_REC) {
						tl = t2;
						L->rec[slot][t2] = (int8_t)kP1;
						L->rec[slot][t2 + 1] = (int8_t)kP1;
						L->rec[slot][t2 + 2] = (int8_t)d;
						if (t2 < F_REC - 3) L->rec[slot][t2 + 3] = 0;
					}
					cur = d;
				}
				last = kP1;
			}
			L->meta[slot] = (uint32_t)votes | ((uint32_t)last << 8) | ((uint32_t)tl << 16) | ((uint32_t)(uint8_t)(int8_t)cur << 24);
		}
		f_sync();
		if (wm) {
			const int nv = f_rd(votes, wl);
			if (maxv < nv) maxv = nv;
			done = true;
		}
	}
	if (done) return;
	if (kv < low || kv > high_w || n0 >= F_SPACE) return;
	if (lane == 0) {
		const int slot = (int)r0 * F_SPACE + n0;
		L->pos[slot] = kv;
		L->meta[slot] = 1u | ((uint32_t)kP1 << 8);
		L->cov[slot] = (uint16_t)((uint32_t)off | ((uint32_t)(off + 16) << 8));
		L->rec[slot][0] = L->rec[slot][1] = (int8_t)kP1;
		L->rec[slot][2] = L->rec[slot][3] = 0;
	}
	if (lane == (int)r0) items = n0 + 1;
	if (maxv == 0) maxv = 1;
	f_sync();
}

// the equal-key run [f, f + c) (absolute item indices) of `key` in bucket b, as gehash_go_q's
// search leaves it (sorted-hashtable.c:760-812): from the 32-byte bucket code (full indexes:
// two selects on its zero bits), from the key-hash record (gapped / small indexes: mid - bwd,
// fwd + bwd), or -- for a bucket the image does not hold (code count byte 255, or keys not sorted)
// -- the literal binary search, back to the first equal key and forward to the last
__device__ __forceinline__ void go_run(const DevIndex &x, uint32_t key, uint32_t b, uint32_t &f, uint32_t &c, bool literal)
{
	const uint32_t q = key / x.nb;
	f = 0;
	c = 0;
	if (literal) {
	} else if (x.bcode) {
		const uint4 *c4 = x.bcode + 2 * (size_t)b;
		const uint4 u0 = c4[0], u1 = c4[1];
		const uint32_t n = u0.y & 255u;
		if (n != 255u) {
			if (n) {
				const uint64_t z[4] = {~(((uint64_t)u0.y << 32) | u0.x) & ~0xffffffffffull, ~(((uint64_t)u0.w << 32) | u0.z),
				                       ~(((uint64_t)u1.y << 32) | u1.x), ~(((uint64_t)u1.w << 32) | u1.z)};
				const int k = (int)q;
				const int fe = k ? code_zero(z, k - 1) - 40 - (k - 1) : 0;
				const int ee = code_zero(z, k) - 40 - k;
				if (ee > fe) { f = u0.x + (uint32_t)fe; c = (uint32_t)(ee - fe); }
			}
			return;
		}
	} else if (x.khash && x.ksorted && q <= 0xffffu && ((x.ksorted[b >> 5] >> (b & 31u)) & 1u)) {
		uint2 rec;
		const bool hit = khash_find(x, key, rec);
		if (!hit) return;
		{
			const uint32_t fwd = rec.y & 0xffffu, bwd = rec.y >> 16;
			f = rec.x - bwd;
			c = fwd + bwd;
			return;
		}
	}
	const int16_t k16 = (int16_t)q;
	const uint32_t first = x.bstart[b];
	const int n = (int)(x.bstart[b + 1] - first);
	const int16_t *KK = x.keys + first;
	if (n) {
		int lo = 0, hi = n - 1, idx;
		bool hit = false;
		for (;;) {
			idx = (lo + hi) / 2;
			const int16_t kk = KK[idx];
			if (kk > k16) hi = idx - 1;
			else if (kk < k16) lo = idx + 1;
			else { hit = true; break; }
			if (hi < lo) break;
		}
		if (hit) {
			while (idx && KK[idx - 1] == k16) idx--;
			int e = idx;
			while (e < n && KK[e] == k16) e++;
			f = first + (uint32_t)idx;
			c = (uint32_t)(e - idx);
		}
	}
}

__global__ void __launch_bounds__(64) fragile_kernel(FParams fp)
{
	__shared__ FLDS L_;
	FLDS *L = &L_;
	const int lane = f_lane();
	const DevIndex &x = fp.ix;
	const int gap = x.gap;
	for (uint32_t jn = blockIdx.x; jn < fp.n_jobs; jn += gridDim.x) {
		const FJob J = fp.jobs[jn];
		const int wl = J.wl, rl = J.rl;
		// ---- the window of the strand's text
		for (int i = lane; i < wl + 1; i += 64) {
			char c = 0;
			if (i < wl) {
				const int p = J.cursor + i;
				c = J.strand ? f_comp(fp.text[J.text + (uint64_t)(rl - 1 - p)]) : fp.text[J.text + (uint64_t)p];
			}
			L->text[i] = c;
		}
		f_sync();
		// ---- probes: subreads k = 0.. until the next one's last offset reaches wl - 16
		int K = 0;
		while (K + 1 < F_STEPS) {
			int o1 = fp.f3[K + 1];
			o1 = o1 - o1 % gap + gap - 1;
			if (o1 >= wl - 16) break;
			K++;
		}
		const int np = (K + 1) * gap;   // <= F_MAXP (checked on the host)
		uint32_t cnt = 0;
		if (lane < np) {
			const int k = lane / gap, i = lane - k * gap;
			int off = fp.f3[k];
			off -= off % gap - i;
			uint32_t key = 0;
			for (int q = 0; q < 16; q++) key |= f_b2i(L->text[off + q]) << (30 - 2 * q);
			// gehash_go_q (sorted-hashtable.c:760-795): binary search, then back to the first equal key
			// and forward over the run -- in a bucket whose keys are sorted, exactly the bucket's whole
			// equal-key run, which the vote path's probe images hold (go_run)
			const uint32_t b = key % x.nb;
			uint32_t f0 = 0;
			go_run(x, key, b, f0, cnt, fp.literal != 0);
			L->pfirst[lane] = f0;
			L->pcnt[lane] = cnt;
			L->ppk[lane] = (uint16_t)((k + 1) | (off << 6));
		}
		// candidate prefix over the probes (probe order)
		{
			uint32_t v = lane < np ? cnt : 0u;
			for (int o = 1; o < 64; o <<= 1) { const uint32_t t = __shfl_up(v, o); if (lane >= o) v += t; }
			if (lane < np) L->pcum[lane + 1] = v;
			if (lane == 0) L->pcum[0] = 0;
		}
		f_sync();
		const uint32_t total = L->pcum[np];
		// ---- vote: chunks of 64 candidates, values loaded lane-parallel, voted in order
		int items = 0, maxv = 0;
		const uint32_t high_w = fp.high - (uint32_t)rl - (uint32_t)wl;
		for (uint32_t c0 = 0; c0 < total; c0 += 64) {
			const uint32_t c = c0 + (uint32_t)lane;
			uint32_t kv = 0, pk = 0;
			if (c < total) {
				int lo = 0, hi = np - 1;
				while (lo < hi) { const int m = (lo + hi + 1) >> 1; if (L->pcum[m] <= c) lo = m; else hi = m - 1; }
				pk = L->ppk[lo];
				kv = x.vals[L->pfirst[lo] + (c - L->pcum[lo])] - (pk >> 6);
			}
			const int m = total - c0 < 64u ? (int)(total - c0) : 64;
			for (int j = 0; j < m; j++) {
				const uint32_t kvj = (uint32_t)f_rd((int)kv, j), pkj = (uint32_t)f_rd((int)pk, j);
				f_vote(L, items, maxv, kvj, (int)(pkj & 63u), (int)(pkj >> 6), fp.low, high_w);
			}
		}
		// ---- decide: lane = used slot in row-major order
		int rs = lane < F_ROWS ? items : 0;
		for (int o = 1; o < 32; o <<= 1) { const int t = __shfl_up(rs, o); if ((lane & 31) >= o) rs += t; }
		const int U = f_rd(rs, F_ROWS - 1);
		auto slot_of = [&](int f) -> int {
			int row = 0;
			for (int r = 0; r < F_ROWS - 1; r++) row += f_rd(rs, r) <= f;
			// every lane takes part in the cross-lane read (an inactive source lane reads as nothing)
			const int sv = __shfl(rs, row > 0 ? row - 1 : 0);
			return row * F_SPACE + (f - (row ? sv : 0));
		};
		svg_fragile_window W;
		memset(&W, 0, sizeof W);
		W.read = J.read; W.block = (uint8_t)fp.block; W.strand = J.strand; W.end = J.end; W.window = J.window;
		W.start = J.cursor; W.length = (uint16_t)wl;
		// top-vote slots with a second recorder section (core-junction.c:5211-5226), in order
		uint32_t nsel = 0, wbase = 0;
		for (int pass = 0; pass < 2; pass++) {
			uint32_t at = 0;
			for (int f0 = 0; f0 < U; f0 += 64) {
				const int f = f0 + lane;
				const int sl = slot_of(f);   // every lane active (cross-lane reads)
				const bool sel = f < U && (int)(L->meta[sl] & 0xffu) >= maxv && L->rec[sl][3] != 0;
				const unsigned long long bm = __ballot(sel);
				if (pass && sel) {
					const uint32_t o = wbase + at + (uint32_t)__popcll(bm & ((1ull << lane) - 1ull));
					if (o < fp.scap) {
						svg_fragile_slot S;
						S.position = L->pos[sl];
						for (int q = 0; q < 9; q++) S.rec[q] = L->rec[sl][q];
						if (!S.rec[6]) S.rec[7] = S.rec[8] = 0;
						S._pad = 0;
						fp.sout[o] = S;
					}
				}
				at += (uint32_t)__popcll(bm);
			}
			if (!pass) {
				nsel = at;
				uint32_t b = 0;
				if (lane == 0 && nsel) b = atomicAdd(fp.scount, nsel);
				wbase = (uint32_t)__shfl((int)b, 0);
			}
		}
		W.n_slots = (uint16_t)nsel;
		W.first_slot = wbase;
		// select_best_vote: the last slot with the top count
		int fmax = -1;
		for (int f0 = 0; f0 < U; f0 += 64) {
			const int f = f0 + lane;
			const int sl = slot_of(f);
			const int cand = f < U && (int)(L->meta[sl] & 0xffu) == maxv ? f : -1;
			int v = cand;
			for (int o = 32; o; o >>= 1) { const int t = __shfl_xor(v, o); v = t > v ? t : v; }
			if (v > fmax) fmax = v;
		}
		if (fmax >= 0) {
			const int ms = slot_of(fmax);
			const uint32_t max_pos = L->pos[ms];
			const int max_cs = (int)(L->cov[ms] & 0xffu), max_ce = (int)(L->cov[ms] >> 8);
			const int c1a = f_locate(x, max_pos + (uint32_t)wl), c1b = f_locate(x, max_pos);
			// core_select_best_matching_halves_maxone: the largest test value, ties to the later slot
			long long best = -1;
			for (int f0 = 0; f0 < U; f0 += 64) {
				const int f = f0 + lane;
				const int sl = slot_of(f);
				long long key = -1;
				if (f < U) {
					const int cs = (int)(L->cov[sl] & 0xffu), ce = (int)(L->cov[sl] >> 8);
					const int os = max_cs > cs ? max_cs : cs, oe = max_ce < ce ? max_ce : ce;
					const uint32_t P = L->pos[sl];
					const int ad = abs((int)((long long)P - (long long)max_pos));
					const int votes = (int)(L->meta[sl] & 0xffu);
					bool ok = oe - os < 14 && ad >= 6 && maxv >= 1 && votes >= 1;
					if (ok) {
						int c1, c2;
						if ((cs < max_cs) + (int)J.strand == 1) { c1 = c1a; c2 = f_locate(x, P); }
						else { c1 = c1b; c2 = f_locate(x, P + (uint32_t)wl); }
						ok = c1 == c2 && ad <= 500000;
					}
					if (ok) key = ((long long)(8888888 + votes * 1000000 - ad) << 12) | f;
				}
				for (int o = 32; o; o >>= 1) { const long long t = __shfl_xor(key, o); key = t > key ? t : key; }
				if (key > best) best = key;
			}
			const int selected = best >= 0 ? (int)(best >> 12) : -1;
			if (selected + maxv * 1000000 > 1000000 && best >= 0) {
				const int s2 = slot_of((int)(best & 4095));
				const int cs = (int)(L->cov[s2] & 0xffu), ce = (int)(L->cov[s2] >> 8);
				const int sp = (((cs < max_cs) ? ce : max_ce) + ((cs < max_cs) ? max_cs : cs)) / 2;
				const uint32_t p2 = L->pos[s2];
				const int v2 = (int)(L->meta[s2] & 0xffu);
				if (sp > 0 && maxv >= 1 && v2 >= 1) {
					// core13_test_donor(window, wl, min, max, sp, strand, wl / 4, ...): lane = split point
					const uint32_t pos1 = max_pos < p2 ? max_pos : p2, pos2 = max_pos < p2 ? p2 : max_pos;
					const int range = wl / 4, rev = J.strand;
					int start = sp - range, end = sp + range;
					if (start < 10) start = 10;
					if (end > wl - 10) end = wl - 10;
					long long bk = -1;   // score << 32 | (0xffff - x) << 1 | gtag: the first best split point
					for (int x0 = start; x0 < end; x0 += 64) {
						const int xx = x0 + lane;
						long long k = -1;
						if (xx < end) {
							char a0, a1, b0, b1;
							f_2base(x, pos1 + (uint32_t)xx, rev, a0, a1);
							f_2base(x, pos2 - 2 + (uint32_t)xx, rev, b0, b1);
							if (!(a0 == b0 && a1 == b1) && f_donor_part(a0, a1) && f_donor_part(b0, b1) && f_paired(a0, a1, b0, b1, rev)) {
								const int bph = rev ? wl - xx : xx;
								int conf = bph < 17 ? bph : 17;
								if (wl - bph < conf) conf = wl - bph;
								int m1, m2, x1, x2;
								if (rev) {
									const uint32_t fe = pos2 + (uint32_t)xx, ss = pos1 + (uint32_t)xx;
									m1 = f_match(x, L->text + bph - conf, fe, conf, 1);
									m2 = f_match(x, L->text + bph, ss - (uint32_t)conf, conf, 1);
									x1 = f_match(x, L->text + bph, fe - (uint32_t)conf, conf, 1);
									x2 = f_match(x, L->text + bph - conf, ss, conf, 1);
								} else {
									const uint32_t fe = pos1 + (uint32_t)xx, ss = pos2 + (uint32_t)xx;
									m1 = f_match(x, L->text + bph - conf, fe - (uint32_t)conf, conf, 0);
									m2 = f_match(x, L->text + bph, ss, conf, 0);
									x1 = f_match(x, L->text + bph, fe, conf, 0);
									x2 = f_match(x, L->text + bph - conf, ss - (uint32_t)conf, conf, 0);
								}
								if (m1 >= conf - 1 && m2 >= conf - 1 && x1 < conf - 3 && x2 < conf - 3) {
									const int score = 3000 - (x1 + x2) + (m1 + m2);
									const int gt = 1 == (rev + (a0 == 'G' || a1 == 'G'));
									k = ((long long)score << 32) | ((long long)(0xffff - xx) << 1) | (long long)gt;
								}
							}
						}
						for (int o = 32; o; o >>= 1) { const long long t = __shfl_xor(k, o); k = t > k ? t : k; }
						if (k > bk) bk = k;
					}
					if (bk >= 0) {
						const int bp = 0xffff - (int)((bk >> 1) & 0xffff);
						const uint32_t a = (uint32_t)bp + max_pos, c = (uint32_t)bp + p2;
						W.junction = 1;
						W.gtag = (uint8_t)(bk & 1);
						W.small_side = (a < c ? a : c) - 1;
						W.large_side = a < c ? c : a;
					}
				}
			}
		}
		if (lane == 0) fp.wout[jn] = W;
		f_sync();
	}
}

// ---------------------------------------------------------------------------------------------- host
static char h_comp(char c)
{
	switch (c) { case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A'; case 'U': return 'A'; }
	return 'N';
}

// the window layout of a read of rl > 160 bases (core-junction.c:5153-5180, the reference's float arithmetic)
static int window_layout(int rl, int *cursor, int *len)
{
	const int windows = rl / F_WIN + 1;
	const float overlap = (1.0 * windows * F_WIN - rl) / (windows - 1);
	for (int ww = 0; ww < windows; ww++) {
		cursor[ww] = (int)(ww * F_WIN - ww * overlap);
		len[ww] = ww == windows - 1 ? rl - cursor[ww] : F_WIN;
	}
	return windows;
}

extern "C" void svg_fragile_free(svg_fragile_result *r)
{
	if (!r) return;
	free(r->windows);
	free(r->slots);
	memset(r, 0, sizeof *r);
}

extern "C" int svg_fragile_batch(svg_index *h, const svg_params *p, const svg_reads *r1, const svg_reads *r2,
                                 svg_fragile_result *out)
{
	if (!h || !p || !r1 || !out) { svg_set_error("svg_fragile_batch: NULL argument"); return SVG_E_ARG; }
	memset(out, 0, sizeof *out);
	if (r2 && r2->n_reads != r1->n_reads) { svg_set_error("svg_fragile_batch: R1/R2 read counts differ"); return SVG_E_ARG; }
	if (!p->do_breakpoint_detection) return 0;   // do_voting runs it for subjunc only
	const int ends = r2 ? 2 : 1;
	const uint64_t n = r1->n_reads;
	// the long read ends' fetched texts (the -S reversal applied: reverse_read, input-files.c:1113)
	std::vector<char> text;
	std::vector<uint64_t> toff((size_t)n * ends, UINT64_MAX);
	std::vector<uint16_t> tlen((size_t)n * ends, 0);
	for (uint64_t r = 0; r < n; r++)
		for (int e = 0; e < ends; e++) {
			const svg_reads *rr = e ? r2 : r1;
			int rl = rr->lens[r] > SVG_READ_KEEP ? SVG_READ_KEEP : rr->lens[r];
			if (rl <= 160) continue;
			const char *s = rr->seq + rr->offsets[r];
			const uint64_t o = text.size();
			text.resize(o + (size_t)rl);
			if (e ? p->reverse_r2 : p->reverse_r1)
				for (int i = 0; i < rl; i++) text[o + (size_t)i] = h_comp(s[rl - 1 - i]);
			else memcpy(&text[o], s, (size_t)rl);
			toff[r * ends + (uint64_t)e] = o;
			tlen[r * ends + (uint64_t)e] = (uint16_t)rl;
		}
	if (text.empty()) return 0;
	// windows of one block, in (read, strand, end, window) order
	std::vector<FJob> jobs;
	for (uint64_t r = 0; r < n; r++)
		for (int s = 0; s < 2; s++)
			for (int e = 0; e < ends; e++) {
				const uint64_t q = r * ends + (uint64_t)e;
				if (toff[q] == UINT64_MAX) continue;
				int cur[SVG_MAX_READ_LENGTH / F_WIN + 2], len[SVG_MAX_READ_LENGTH / F_WIN + 2];
				const int nw = window_layout(tlen[q], cur, len);
				for (int w = 0; w < nw; w++) {
					FJob J;
					J.text = toff[q]; J.read = (uint32_t)r; J.rl = tlen[q]; J.cursor = (uint16_t)cur[w];
					J.wl = (uint16_t)len[w]; J.strand = (uint8_t)s; J.end = (uint8_t)e; J.window = (uint8_t)w; J.pad = 0;
					if (len[w] > F_MAXW - 8) { svg_set_error("fragile window of %d bases", len[w]); return SVG_E_UNSUPPORTED; }
					jobs.push_back(J);
				}
			}
	int16_t f3[F_STEPS];
	{
		const float step = 3.00001f;
		for (int k = 0; k < F_STEPS; k++) f3[k] = (int16_t)(int)(step * k);
	}
	{
		// the kernel holds a window's probes in one wave: (subreads) x gap <= 64
		int wmax = 0;
		for (const FJob &J : jobs) wmax = J.wl > wmax ? J.wl : wmax;
		for (int b = 0; b < h->nblocks; b++) {
			const int gap = (b ? h->blk[b] : h)->dix.gap;
			int K = 0;
			while (K + 1 < F_STEPS) { int o1 = f3[K + 1]; o1 = o1 - o1 % gap + gap - 1; if (o1 >= wmax - 16) break; K++; }
			if ((K + 1) * gap > F_MAXP) { svg_set_error("fragile windows need %d probes", (K + 1) * gap); return SVG_E_UNSUPPORTED; }
		}
	}
	HIPCHK(hipSetDevice(h->device));
	hipStream_t st = h->stream;
	if (h->last_pending) HIPCHK(hipStreamWaitEvent(st, h->ev_last, 0));
	const uint64_t nj = jobs.size(), nwin = nj * (uint64_t)h->nblocks;
	char *d_text = NULL;
	FJob *d_jobs = NULL;
	int16_t *d_f3 = NULL;
	svg_fragile_window *d_w = NULL;
	svg_fragile_slot *d_s = NULL;
	uint32_t *d_cnt = NULL;
	int rc = 0;
	std::vector<svg_fragile_slot> slots;
	out->windows = (svg_fragile_window *)malloc(sizeof(svg_fragile_window) * nwin);
	if (!out->windows) { svg_set_error("out of host memory"); return SVG_E_NOMEM; }
	out->n_windows = nwin;
	uint32_t scap = (uint32_t)(nj < (1u << 20) ? nj * 2 + 1024 : nj);
	if ((rc = dmalloc(h, (void **)&d_text, text.size() + 64)) || (rc = dmalloc(h, (void **)&d_jobs, sizeof(FJob) * nj)) ||
	    (rc = dmalloc(h, (void **)&d_f3, sizeof f3)) || (rc = dmalloc(h, (void **)&d_w, sizeof(svg_fragile_window) * nj)) ||
	    (rc = dmalloc(h, (void **)&d_cnt, 64)))
		goto done;
	if (hipMemcpyAsync(d_text, text.data(), text.size(), hipMemcpyHostToDevice, st) != hipSuccess ||
	    hipMemcpyAsync(d_jobs, jobs.data(), sizeof(FJob) * nj, hipMemcpyHostToDevice, st) != hipSuccess ||
	    hipMemcpyAsync(d_f3, f3, sizeof f3, hipMemcpyHostToDevice, st) != hipSuccess) {
		svg_set_error("svg_fragile_batch: upload failed"); rc = SVG_E_DEVICE; goto done;
	}
	for (int b = 0; b < h->nblocks && !rc; b++) {
		const svg_index *bk = b ? h->blk[b] : h;
		bool stored = false;
		for (int attempt = 0; attempt < 2 && !rc; attempt++) {
			if (!d_s && (rc = dmalloc(h, (void **)&d_s, sizeof(svg_fragile_slot) * (size_t)scap))) break;
			FParams fp;
			memset(&fp, 0, sizeof fp);
			fp.ix = bk->dix; fp.text = d_text; fp.jobs = d_jobs; fp.n_jobs = (uint32_t)nj; fp.block = b; fp.f3 = d_f3;
			fp.low = bk->dix.start_base_offset; fp.high = bk->dix.start_base_offset + bk->dix.length;
			fp.wout = d_w; fp.sout = d_s; fp.scount = d_cnt; fp.scap = scap;
			fp.literal = svg_get_option("keys_literal") != 0;
			uint64_t grid = (uint64_t)h->n_cu * 5;
			if (grid > nj) grid = nj;
			if (hipMemsetAsync(d_cnt, 0, 4, st) != hipSuccess) { rc = SVG_E_DEVICE; break; }
			hipLaunchKernelGGL(fragile_kernel, dim3((unsigned)grid), dim3(64), 0, st, fp);
			if (hipGetLastError() != hipSuccess) { svg_set_error("fragile_kernel launch failed"); rc = SVG_E_DEVICE; break; }
			uint32_t used = 0;
			if (hipMemcpyAsync(&used, d_cnt, 4, hipMemcpyDeviceToHost, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess) {
				svg_set_error("fragile_kernel failed"); rc = SVG_E_DEVICE; break;
			}
			if (used > scap) {   // more reported slots than room: once more with room for all
				hipFree(d_s);
				d_s = NULL;
				scap = used + 1024;
				continue;
			}
			std::vector<svg_fragile_slot> s(used);
			svg_fragile_window *wo = out->windows + (uint64_t)b * nj;
			if ((used && hipMemcpy(s.data(), d_s, sizeof(svg_fragile_slot) * used, hipMemcpyDeviceToHost) != hipSuccess) ||
			    hipMemcpy(wo, d_w, sizeof(svg_fragile_window) * nj, hipMemcpyDeviceToHost) != hipSuccess) {
				svg_set_error("svg_fragile_batch: download failed"); rc = SVG_E_DEVICE; break;
			}
			// slots in window order (the kernel appends them in completion order)
			for (uint64_t j = 0; j < nj; j++) {
				svg_fragile_window *W = &wo[j];
				const uint32_t f = W->first_slot;
				W->first_slot = (uint32_t)slots.size();
				for (uint32_t q = 0; q < W->n_slots; q++) slots.push_back(s[f + q]);
			}
			stored = true;
			break;
		}
		// the second attempt has room for every slot the first one counted; a block that still was
		// not stored is an error, never a silently unwritten window range
		if (!rc && !stored) {
			svg_set_error("svg_fragile_batch: block %d: reported slots exceed the retried capacity", b);
			rc = SVG_E_DEVICE;
		}
	}
done:
	hipFree(d_text); hipFree(d_jobs); hipFree(d_f3); hipFree(d_w); hipFree(d_s); hipFree(d_cnt);
	if (rc) { svg_fragile_free(out); return rc; }
	out->n_slots = slots.size();
	out->slots = (svg_fragile_slot *)malloc(sizeof(svg_fragile_slot) * (slots.size() + 1));
	if (!out->slots) { svg_fragile_free(out); svg_set_error("out of host memory"); return SVG_E_NOMEM; }
	if (!slots.empty()) memcpy(out->slots, slots.data(), sizeof(svg_fragile_slot) * slots.size());
	return 0;
}
