// svg_vote.hip -- MI355X (gfx950) seed-and-vote kernel + the C ABI of include/subread_vote.h
//
// One wavefront (64 lanes) owns one read (SE) or one read pair (PE) at a time
// and walks the reference's voting step for it:
//
//   phase P  (lanes = probes)    every 16-mer of both strands of every end is
//            packed from the read text in LDS (genekey2int, input-files.c:1232),
//            hashed to its bucket (key % nb) and binary-searched in HBM exactly
//            like gehash_go_X (sorted-hashtable.c:947-981); each lane keeps the
//            search midpoint and the length of the equal-key run on both sides.
//            All probes of a read are in flight together, so the dependent
//            HBM chain (bucket bounds -> keys -> run) is paid once per read.
//   phase G  (lanes = candidates) the hit values of one (strand, end) are
//            gathered into an LDS queue in the reference's visiting order:
//            subread_no, then xk1, then mid..last, then mid-1..first
//            (sorted-hashtable.c:1109-1119).
//   phase V  (lanes = vote slots) the queue is replayed in order.  For each
//            candidate the lanes test the <=24 slots of the rows (kv+iix)/5 %30,
//            iix = 0,+5,-5 (sorted-hashtable.c:995-1001) in parallel; a ballot
//            finds, in row/slot order, every slot within the indel tolerance,
//            each matched lane applies its own shift-indel mark and toli
//            roll-back (sorted-hashtable.c:1021-1039) up to the first slot that
//            actually takes the vote, and that lane votes (:1041-1068).  With
//            no taker a new slot is opened in row kv/5 %30 (:1071-1106).
//   phase K  (lanes = slots / pairs) top-3 distinct vote values, candidate
//            lists, PE pair scoring and the final <=multi_best records
//            (process_voting_junction_PE_topK, core-junction.c:2199-2530).
//
// The vote table keeps the reference's geometry (30 rows x 24 slots, first
// match wins, 24-slot cap) so that overflow and tie behaviour are identical.
// Hot slot state (position + packed votes/last/toli/shift/cursor) lives in LDS;
// the cold part (coverage start/end, 21-entry indel recorder) lives in a
// per-wave HBM scratch that stays L2-resident.  Integer work only: no MFMA.
#include <hip/hip_runtime.h>
#include <string>
#include <vector>
#include <chrono>
#include <atomic>
#include <deque>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <pthread.h>
#include <sys/mman.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <stdio.h>
#include "subread_vote.h"
#include "svg_internal.h"
#include "svg_device.h"

#define ROWS 30
#define SPACE 24              // GENE_VOTE_SPACE: slots a row may hold
// LDS row stride of the vote table, in slots: 25 x 8 B = 50 dwords, so the rows of the 30-row
// table start on 30 different bank pairs (a 24-slot stride puts every row on one of 4 and made
// batch mode's per-lane random-row scans 8-way bank conflicts).  Slot ids (LDS index, cold state,
// top-K handles) are row * PSTR + slot.
#define PSTR 25
#define NSLOT (ROWS * PSTR)
#define REC_LEN 21
#define COLD_WORDS 8          // per slot: cs|ce<<16, rec[21] as bytes, pad
#define JCW 17

// ---------------------------------------------------------------------------------------------
// LDS layout of one wave.  Row occupancy (items[30]) and max_vote live in
// registers (lane 32*end+row holds items[row]); only slot state is in LDS.
#define CAND_CAP 64
template <int ENDS, int MAXL, int MAXP, bool SJ>
struct WaveLDS {
	static constexpr int MAXS = ENDS == 1 ? 16 : 64;   // max_vote_simples capacity
	// One physical vote table (gene_vote_t, [row*24+slot]): x = position, y = meta =
	// votes | last<<8 | (toli | shift<<7)<<16 | (u8)cursor<<24.  PE votes end 0 first, then
	// compacts its used slots (flattened row order, the order every top-K scan uses) into
	// cl/cls and votes end 1 in the same table.
	static constexpr int CAPL = ENDS == 2 ? 64 : 1;
	uint2 pm[NSLOT];
	uint2 cl[CAPL];                       // end 0 compacted: position, meta (entries >= CAPL: HBM)
	uint16_t cls[CAPL];                   // end 0 compacted: table slot (cold-state index)
	uint32_t pmid[ENDS][2][MAXP];         // probe: binary-search midpoint (absolute item index)
	uint16_t pfwd[ENDS][2][MAXP];         // equal-key items at mid..last
	uint16_t pbwd[ENDS][2][MAXP];         // equal-key items at first..mid-1
	uint32_t pcum[MAXP + 1];              // candidate prefix of the (strand,end) being replayed
	uint32_t res[ENDS][3][17];            // the read's stored mapping_result_t (68 B)
	uint32_t tmp[ENDS][3][17];            // top-K output under construction
	uint32_t jres[SJ ? ENDS : 1][3][4];   // subjunc_result_t (subjunc variants only)
	uint32_t jtmp[SJ ? ENDS : 1][3][4];
	uint32_t simp_pos[ENDS][MAXS];        // simple_mapping_t: position
	uint16_t simp_slot[ENDS][MAXS];       // slot index, or 0x8000|stored index
	uint16_t simp_votes[ENDS][MAXS];
	int32_t simp_loc[ENDS == 2 ? 2 : 1][ENDS == 2 ? MAXS : 1];   // PE: locate_gene_position of each simple (position)
	int16_t simp_chr[ENDS == 2 ? 2 : 1][ENDS == 2 ? MAXS : 1];   //     its chromosome, -1 where locate fails
	uint16_t bm[SJ ? ENDS : 1][10];
	uint8_t rnew[32];                     // batch mode: new row occupancy (0xff = unchanged)
	alignas(16) unsigned long long btab[32];   // batch mode: lane masks of the chunk's candidates by kv bin, then by row
	uint8_t gwin[SJ ? 2 : 1][SJ ? 64 : 4];   // subjunc donor windows of the .array
	char text[SJ ? ENDS : 1][2][SJ ? MAXL : 4];   // strand 0 / strand 1 (reverse_read) form, donor scoring only
};

// ---------------------------------------------------------------------------------------------
// wave helpers
__device__ __forceinline__ int lane_id() { return __lane_id(); }
__device__ __forceinline__ unsigned long long ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int lanes_below(unsigned long long m) { return __popcll(m & ((1ull << lane_id()) - 1ull)); }
__device__ __forceinline__ void wsync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); __builtin_amdgcn_wave_barrier(); }
__device__ __forceinline__ int wave_max(int v)
{
	for (int o = 32; o; o >>= 1) { int t = __shfl_xor(v, o); v = t > v ? t : v; }
	return v;
}
__device__ __forceinline__ int wave_min(int v)
{
	for (int o = 32; o; o >>= 1) { int t = __shfl_xor(v, o); v = t < v ? t : v; }
	return v;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v)
{
	for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
	return v;
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
	int l = lane_id();
	for (int o = 1; o < 64; o <<= 1) { uint32_t t = __shfl_up(v, o); if (l >= o) v += t; }
	return v;
}

// base2int, subread.h:238
__device__ __forceinline__ uint32_t b2i(char c) { return c < 'G' ? (c == 'A' ? 0u : 2u) : (c == 'G' ? 1u : 3u); }
// reverse_read table, input-files.c:1111 (ASCII; everything else -> 'N')
__device__ __forceinline__ char comp(char c)
{
	return c == 'A' ? 'T' : c == 'C' ? 'G' : c == 'G' ? 'C' : (c == 'T' || c == 'U') ? 'A' : 'N';
}

// meta packing: votes [0,7) | last [7,14) | shift [14] | x [15,17) | spill [17] | then
//   unspilled: first [18,25) | fx [25,27)      spilled: toli [18,23) | cursor [23,29) (signed)
// votes and last (a subread number + 1) are <= 64 (applied subreads).  x / fx: the gap slot of the
// last / first vote, so coverage_end (last vote's offset + 16) and coverage_start (first vote's
// offset) follow from the meta.  Until a slot opens its first indel section its recorder is
// (first, last, 0) with toli = cursor = 0 (sorted-hashtable.c:1049-1063,1096-1102) and it has no
// cold state at all; the first section spills coverage_start and the recorder to the cold scratch
// (HBM), and the same bits then hold toli and cursor.
#define M_SPILL (1u << 17)
__device__ __forceinline__ int m_votes(uint32_t m) { return m & 0x7f; }
__device__ __forceinline__ int m_last(uint32_t m) { return (m >> 7) & 0x7f; }
__device__ __forceinline__ int m_shift(uint32_t m) { return (m >> 14) & 1; }
__device__ __forceinline__ int m_x(uint32_t m) { return (m >> 15) & 3; }
__device__ __forceinline__ bool m_spilled(uint32_t m) { return (m & M_SPILL) != 0; }
__device__ __forceinline__ int m_first(uint32_t m) { return (m >> 18) & 0x7f; }
__device__ __forceinline__ int m_fx(uint32_t m) { return (m >> 25) & 3; }
__device__ __forceinline__ int m_toli(uint32_t m) { return m_spilled(m) ? (int)((m >> 18) & 31u) : 0; }
__device__ __forceinline__ int m_cursor(uint32_t m) { return m_spilled(m) ? ((int)(m << 3)) >> 26 : 0; }
// a spilled slot's meta
__device__ __forceinline__ uint32_t m_pack_s(int votes, int last, int shift, int x, int toli, int cursor)
{
	return (uint32_t)(votes & 0x7f) | ((uint32_t)(last & 0x7f) << 7) | ((uint32_t)shift << 14) | ((uint32_t)x << 15) | M_SPILL |
	       ((uint32_t)(toli & 31) << 18) | (((uint32_t)cursor & 63u) << 23);
}
// an unspilled slot's meta
__device__ __forceinline__ uint32_t m_pack_u(int votes, int last, int shift, int x, int first, int fx)
{
	return (uint32_t)(votes & 0x7f) | ((uint32_t)(last & 0x7f) << 7) | ((uint32_t)shift << 14) | ((uint32_t)x << 15) |
	       ((uint32_t)(first & 0x7f) << 18) | ((uint32_t)fx << 25);
}
// the gap slot of a subread offset (off = base - base % gap + x; gap 1 (-F) or 3 (default))
__device__ __forceinline__ int gap_x(int off, int gap) { return gap == 1 ? 0 : off % gap; }

// record field offsets in mapping_result_t (byte offsets)
#define MR_POS 0
#define MR_FLAGS 4
#define MR_VOTES 8
#define MR_USED 10
#define MR_NONINF 12
#define MR_INDELS 13
#define MR_REC 16
#define MR_CS 60
#define MR_CE 62

__device__ __forceinline__ uint32_t abs32u(uint32_t x) { return x > 0x7fffffffu ? (0xffffffffu - x) + 1 : x; }
__device__ __forceinline__ int16_t rec_votes(const uint32_t *r) { return (int16_t)(r[2] & 0xffff); }
__device__ __forceinline__ uint32_t rec_pos(const uint32_t *r) { return r[0]; }
__device__ __forceinline__ void rec_set_votes(uint32_t *r, int v) { r[2] = (r[2] & 0xffff0000u) | ((uint32_t)v & 0xffff); }
__device__ __forceinline__ int rec_used(const uint32_t *r) { return (int16_t)(r[2] >> 16); }
__device__ __forceinline__ void rec_set_used(uint32_t *r, int v) { r[2] = (r[2] & 0xffffu) | ((uint32_t)v << 16); }
__device__ __forceinline__ int rec_noninf(const uint32_t *r) { return r[3] & 0xff; }
__device__ __forceinline__ void rec_set_noninf(uint32_t *r, int v) { r[3] = (r[3] & 0xffffff00u) | ((uint32_t)v & 0xff); }
__device__ __forceinline__ int rec_cs(const uint32_t *r) { return r[15] & 0xffff; }

// ---------------------------------------------------------------------------------------------
// cold per-slot state in HBM scratch, spilled slots only: word 0 = coverage_start, bytes 4..24 =
// indel recorder
__device__ __forceinline__ uint32_t *cold_slot(uint32_t *cold, int slot) { return cold + slot * COLD_WORDS; }
__device__ __forceinline__ int cold_rec(const uint32_t *cs, int i) { return (int)((const int8_t *)(cs + 1))[i]; }
__device__ __forceinline__ void cold_set_rec(uint32_t *cs, int i, int v) { ((int8_t *)(cs + 1))[i] = (int8_t)v; }

// ---------------------------------------------------------------------------------------------
// per-read context (registers, wave-uniform values)
struct ReadCtx {
	int rl[2];
	int applied[2];
	int step[2];
	int np[2];          // probes per strand for each end (applied*gap)
};

#ifdef SVG_STAMPS
#define STAMP(k) do { unsigned long long _t = __builtin_amdgcn_s_memtime(); acc[k] += _t - t_last; t_last = _t; } while (0)
#else
#define STAMP(k) do { } while (0)
#endif

template <int ENDS, int MAXL, int MAXP, bool SJ>
struct Wave {
#ifdef SVG_STAMPS
	unsigned long long t_last, acc[12];   // [8..11]: phase K split (top-3, simples, pairs, emission)
	unsigned long long why[4];   // batch mode's serial candidates by reason (stats[28..31])
#endif
	WaveLDS<ENDS, MAXL, MAXP, SJ> *L;
	uint32_t *cold[2];      // [ENDS] cold slot state
	uint32_t *shift_locs[2];
	const KParams *kp;
	ReadCtx rc;
	int items_v;            // lane 32*e + r: items[r] of table e (gene_vote_t.items)
	int max_vote[2];        // gene_vote_t.max_vote per table (wave-uniform)
	int nshift[2];          // shift_indel_NO per table (wave-uniform)
	uint32_t *ovf;          // PE: compacted end-0 entries beyond the LDS list (HBM scratch)
	uint32_t wb[2];         // subjunc: first .array byte of the left / right donor window
	int cur_strand;

	__device__ __forceinline__ static int rd(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
	// a per-end register array read at a run-time end (PE top-K / junction search): a select, since
	// one dynamic index puts the whole Wave object -- and the kernel's KParams copy -- in scratch
	template <class T> __device__ __forceinline__ static T end_sel(const T (&a)[2], int e)
	{
		const T a0 = a[0], a1 = a[1];   // (values, not `e ? a[1] : a[0]`: that is a select of two addresses)
		return e ? a1 : a0;
	}

	// ---------------------------------------------------------------- probe offset of probe p
	__device__ __forceinline__ int probe_off(int e, int p) const
	{
		int gap = kp->ix.gap;
		if (gap == 1) return (int)(((int64_t)end_sel(rc.step, e) * p) >> 16);   // full index: no division (gap is uniform)
		int k = p / gap, x = p - k * gap;
		int off = (int)(((int64_t)end_sel(rc.step, e) * k) >> 16);
		if (gap > 1) off -= off % gap - x;
		return off;
	}

	// offset of subread kP1 - 1 at gap slot x (core.c:3169-3171)
	__device__ __forceinline__ int sub_off(int e, int kP1, int x) const
	{
		const int gap = kp->ix.gap;
		int off = (int)(((int64_t)end_sel(rc.step, e) * (kP1 - 1)) >> 16);
		if (gap > 1) off -= off % gap - x;
		return off;
	}
	// confident_coverage_start | confident_coverage_end << 16 of a slot (meta M)
	__device__ __forceinline__ uint32_t slot_cw(int e, int slot, uint32_t M) const
	{
		const int ce = sub_off(e, m_last(M), m_x(M)) + 16;
		const int cs = m_spilled(M) ? (int)(cold_slot(end_sel(cold, e), slot)[0] & 0xffffu) : sub_off(e, m_first(M), m_fx(M));
		return (uint32_t)(uint16_t)cs | ((uint32_t)(uint16_t)ce << 16);
	}
	// indel recorder entry i of a slot (meta M)
	__device__ __forceinline__ int slot_rec(int e, int slot, uint32_t M, int i) const
	{
		if (m_spilled(M)) return cold_rec(cold_slot(end_sel(cold, e), slot), i);
		return i == 0 ? m_first(M) : (i == 1 ? m_last(M) : 0);
	}

	// ---------------------------------------------------------------- vote-table reset (init_gene_vote)
	template <int E>
	__device__ __forceinline__ void table_reset()
	{
		if ((lane_id() >> 5) == E) items_v = 0;
		max_vote[E] = 0;
	}

	// one group of <= 64 candidate slots, lanes in the reference's scan order
	// (rows iix = 0,+5,-5,..., slots ascending).  Returns true when a slot took the vote.
	template <int E>
	__device__ __forceinline__ bool vote_group(bool valid, int slot, uint32_t kv, int kP1, int off, int round)
	{
		const int lane = lane_id();
		const int tol = kp->tol;
		const uint2 pmv = L->pm[valid ? slot : 0];   // unconditional: no exec-mask branch
		const uint32_t P = valid ? pmv.x : 0u, M = valid ? pmv.y : 0u;
		int d = (int)(kv - P);
		int sh = m_shift(M);
		int t = (round > 0 && sh) ? 0 : tol;
		bool match = valid && d >= -t && d <= t;
		unsigned long long mm = ballot(match);
		if (!mm) return false;
		int votes = m_votes(M), last = m_last(M), tl = m_toli(M), cur = m_cursor(M);
		bool sev = match && round == 0 && tl > 0 && d == 0 && !sh;
		bool rb = false;
		if (match && last == kP1 && tl > 0) {    // roll-back test (sorted-hashtable.c:1027-1039); tl > 0: spilled
			const uint32_t *cs = cold_slot(cold[E], slot);
			int md = tl >= 3 ? cold_rec(cs, tl - 1) : 0;
			int nd = md - d;
			md -= cold_rec(cs, tl + 2);
			rb = abs(md) > abs(nd);
		}
		int last2 = rb ? last - 1 : last;
		bool wv = match && !(kP1 <= last2);
		unsigned long long wm = ballot(wv);
		int wl = wm ? (__ffsll((long long)wm) - 1) : 64;
		bool apply = match && lane <= wl;
		unsigned long long smask = ballot(apply && sev);
		if (apply && sev) shift_locs[E][nshift[E] + lanes_below(smask)] = P;
		nshift[E] += __popcll(smask);
		int nvotes = votes;
		if (apply) {
			int nlast = last, ntl = tl, nsh = sh | (sev ? 1 : 0), ncur = cur, nx = m_x(M);
			bool spill = m_spilled(M);
			if (rb) { ntl -= 3; nlast -= 1; nvotes -= 1; }
			if (lane == wl) {
				nvotes += 1;
				// coverage_end = max(coverage_end, off+16): off rises strictly along the probe order
				// of a round (step >= gap<<16), so it is this vote's off+16 -- kept as (last, x)
				nx = gap_x(off, kp->ix.gap);
				if (d == ncur) {
					if (spill) cold_set_rec(cold_slot(cold[E], slot), ntl + 1, kP1);   // implicit: rec[1] = last
				} else if (!spill) {
					// first indel section (toli 0): coverage_start and the recorder go to the cold
					// scratch, rec[0..7] = first, last, 0, kP1, kP1, d, 0, 0
					uint32_t *cs = cold_slot(cold[E], slot);
					cs[0] = (uint32_t)(uint16_t)sub_off(E, m_first(M), m_fx(M));
					cs[1] = (uint32_t)(uint8_t)m_first(M) | ((uint32_t)(uint8_t)last << 8) | ((uint32_t)(uint8_t)kP1 << 24);
					cs[2] = (uint32_t)(uint8_t)kP1 | ((uint32_t)(uint8_t)(int8_t)d << 8);
					ntl = 3;
					ncur = (int)(int8_t)d;
					spill = true;
				} else {
					uint32_t *cs = cold_slot(cold[E], slot);
					int t2 = ntl + 3;
					if (t2 < REC_LEN) {
						ntl = t2;
						cold_set_rec(cs, t2, kP1);
						cold_set_rec(cs, t2 + 1, kP1);
						cold_set_rec(cs, t2 + 2, d);
						if (t2 < REC_LEN - 3) cold_set_rec(cs, t2 + 3, 0);
					}
					ncur = (int)(int8_t)d;
				}
				nlast = kP1;
			}
			L->pm[slot].y = spill ? m_pack_s(nvotes, nlast, nsh, nx, ntl, ncur) : m_pack_u(nvotes, nlast, nsh, nx, m_first(M), m_fx(M));
		}
		wsync();
		if (wm) {
			int nv = rd(nvotes, wl);
			if (max_vote[E] < nv) max_vote[E] = nv;
			return true;
		}
		return false;
	}

	// ---------------------------------------------------------------- phase V: one candidate (gehash_go_X body)
	// candidate packing: kP1 (6 bits) | off << 6 (11) | r0 << 17 | rp << 22 | rm << 27 (5 each),
	// rows of iix = 0, +5, -5 (sorted-hashtable.c:995-1001) computed lane-parallel at gather time
	__device__ static uint32_t cand_pack(uint32_t kv, int kP1, int off)
	{
		uint32_t r0 = (kv / 5u) % ROWS, rp = ((kv + 5u) / 5u) % ROWS, rm = ((kv - 5u) / 5u) % ROWS;
		return (uint32_t)kP1 | ((uint32_t)off << 6) | (r0 << 17) | (rp << 22) | (rm << 27);
	}

	template <int E>
	__device__ void vote_one(uint32_t kv, uint32_t pk, int round, uint32_t high_b)
	{
		const int lane = lane_id();
		const int tol = kp->tol;
		const int kP1 = (int)(pk & 63u), off = (int)((pk >> 6) & 2047u);
		const uint32_t r0 = (pk >> 17) & 31u;
		const int n0 = rd(items_v, E * 32 + (int)r0);
		bool found = false;
		if (kp->ii_end == 5) {
			// rows r0, r0+1, r0-1 (iix = 0, +5, -5) in one LDS round trip, lanes packed over the used
			// slots in the reference's scan order (lane l = the l-th used slot of r0, then rp, then
			// rm; ballot order = scan order).  Rows hold a few slots each (C3 deferred reads: ~4), so
			// the three runs sit in distinct banks -- a fixed 24/24/16 lane map made rp's slots 16-23
			// and rm's 0-7 share banks on every fetch (29% of the kernel's LDS cycles in conflicts).
			// More than 64 used slots (rare): a second group, after the first found nothing.
			const uint32_t rp = (pk >> 22) & 31u, rm = pk >> 27;
			const int np_ = rd(items_v, E * 32 + (int)rp), nm = rd(items_v, E * 32 + (int)rm);
			const int tot = n0 + np_ + nm;
			for (int g = 0; g < tot && !found; g += 64) {
				const int l = g + lane;
				const bool in0 = l < n0, in1 = !in0 && l < n0 + np_;
				const uint32_t row = in0 ? r0 : (in1 ? rp : rm);
				const int sl = in0 ? l : (in1 ? l - n0 : l - n0 - np_);
				found = vote_group<E>(l < tot, (int)row * PSTR + sl, kv, kP1, off, round);
			}
		} else {
			for (int iix = 0; iix <= kp->ii_end && !found; iix = iix > 0 ? -iix : (-iix + 5)) {
				uint32_t r = iix ? ((kv + (uint32_t)iix) / 5u) % ROWS : r0;
				int cnt = iix ? rd(items_v, E * 32 + (int)r) : n0;
				if (!cnt) continue;
				found = vote_group<E>(lane < cnt, (int)r * PSTR + lane, kv, kP1, off, round);
			}
		}
		if (!found && kv >= kp->low && kv <= high_b && n0 < SPACE) {
			int sh = 0;
			if (round > 0) {
				bool any = false;
				for (int j = lane; j < nshift[E]; j += 64) {
					uint32_t loc = shift_locs[E][j];
					if (kv >= loc - (uint32_t)tol && kv <= loc + (uint32_t)tol) any = true;
				}
				sh = ballot(any) ? 1 : 0;
			}
			if (lane == 0) {
				// a new slot: recorder (k+1, k+1, 0), coverage off..off+16, all in the meta
				const int x = gap_x(off, kp->ix.gap);
				L->pm[(int)r0 * PSTR + n0] = make_uint2(kv, m_pack_u(1, kP1, sh, x, kP1, x));
			}
			if (lane == E * 32 + (int)r0) items_v = n0 + 1;
			if (max_vote[E] == 0) max_vote[E] = 1;
			wsync();
		}
	}

	// ---------------------------------------------------------------- batch mode (round 0)
	// Lane c holds candidate c of a chunk of m <= 64, in the reference's order.  Two kinds of
	// candidate have an outcome the other candidates of the chunk cannot change:
	//  A (opens a slot): no slot of the table within the tolerance in its three rows (so it finds
	//    nothing), no other chunk candidate within 2*tol (no slot opened in the chunk can match it,
	//    nor its slot theirs), and no earlier serial candidate in its row (so its slot index is its
	//    rank among the row's openers) -- it only opens a slot in row kv/5 %30
	//    (sorted-hashtable.c:1071-1106);
	//  B (votes): exactly one slot s within the tolerance, unspilled (toli 0: no roll-back, no
	//    shift-indel mark), matched exactly (d == 0 == its cursor: no indel section) with
	//    kP1 > last(s), every chunk candidate within 2*tol of it a B candidate of the same slot with a
	//    different kP1 -- the chunk's votes on s are then s's whole fold in chunk order
	//    (sorted-hashtable.c:1041-1047: votes += 1, last = kP1, coverage_end from the last), applied
	//    at once by the group's last lane.
	// A and B candidates touch slots no other candidate of the chunk reads, so they are settled
	// together; the rest are left for the serial replay (vote_one, in order).  Returns those lanes.
	template <int E>
	__device__ unsigned long long batch_create(int kvv, int kov, int m, uint32_t high_b)
	{
		const int lane = lane_id();
		const bool act = lane < m;
		const uint32_t kv = (uint32_t)kvv, pk = (uint32_t)kov;
		const int tol = kp->tol, kP1 = (int)(pk & 63u), off = (int)((pk >> 6) & 2047u);
		const uint32_t r0 = (pk >> 17) & 31u, rp = (pk >> 22) & 31u, rm = pk >> 27;
		// row occupancy of the candidate's three rows (every lane active for the shuffles)
		const int n0 = __shfl(items_v, E * 32 + (int)r0), np_ = __shfl(items_v, E * 32 + (int)rp),
		          nm = __shfl(items_v, E * 32 + (int)rm);
		// the table's slots within the tolerance (up to two), the first one's index, meta and offset
		int nmatch = 0, tslot = -1, td = 1;
		uint32_t tM = 0u;
		if (act) {
			// the three rows in scan order, four consecutive slots of a row per LDS round trip (the
			// reads past a row's used slots are masked; the index is clamped to the table)
#pragma unroll
			for (int sg = 0; sg < 3; sg++) {
				const int cnt = sg == 0 ? n0 : (sg == 1 ? np_ : nm);
				const int base = (int)(sg == 0 ? r0 : (sg == 1 ? rp : rm)) * PSTR;
				for (int q = 0; q < cnt && nmatch < 2; q += 4) {
					uint2 e[4];
#pragma unroll
					for (int k = 0; k < 4; k++) e[k] = L->pm[min(base + q + k, NSLOT - 1)];
#pragma unroll
					for (int k = 0; k < 4; k++) {
						const int d = (int)(kv - e[k].x);
						if (q + k < cnt && (uint32_t)(d + tol) <= (uint32_t)(2 * tol)) {
							if (!nmatch) { tslot = base + q + k; tM = e[k].y; td = d; }
							nmatch++;
						}
					}
				}
			}
		}
		if constexpr (!SJ) STAMP(7);   // diagnostics (align variants): the slot scan
		const bool bcand = act && nmatch == 1 && td == 0 && !m_spilled(tM) && kP1 > m_last(tM);
		// chunk neighbours: eqm = the candidates with this kv (this lane included), nbfar = one at
		// 0 < |d| <= 2*tol.  A B candidate's slot position is its kv, so its group (the chunk's
		// votes on the slot) is eqm.  The candidates go into a 62-entry table of lane masks by kv bin
		// (bins of 2^sb >= 2*tol positions, so a candidate within 2*tol is in the same or an adjacent
		// bin, bins counted modulo 2^(32-sb) as the distance test wraps modulo 2^32), and each lane
		// tests only the candidates of its three bins' entries -- a few, where testing all m against
		// all m cost ~100 instructions per 4.  Entries 0-31 are btab, 32-61 the vote table's unused
		// 25th slot of each row (the row stride is 25, a row holds at most 24)
		const int sb = tol < 1 ? 0 : 32 - __clz(2 * tol - 1);
		const uint32_t bin = sb < 32 ? kv >> sb : 0u, bmask = sb < 32 ? 0xffffffffu >> sb : 0u;
		auto nb_ent = [&](uint32_t b) -> unsigned long long * {
			const uint32_t h = (b & bmask) % 62u;
			return h < 32u ? &L->btab[h] : reinterpret_cast<unsigned long long *>(&L->pm[(int)(h - 32u) * PSTR + SPACE]);
		};
		if (lane < 62) *nb_ent((uint32_t)lane) = 0ull;   // (bmask >= 63: sb <= 26, tol < 2^25)
		wsync();
		if (act) atomicOr(nb_ent(bin), 1ull << lane);
		wsync();
		unsigned long long near = act ? (*nb_ent(bin - 1u) | *nb_ent(bin) | *nb_ent(bin + 1u)) & ~(1ull << lane) : 0ull;
		bool nbfar = false;
		unsigned long long eqm = act ? 1ull << lane : 0ull;
		while (ballot(near != 0ull)) {   // (every lane takes part in the shuffle; no branches inside)
			const bool has = near != 0ull;
			const int j = has ? __ffsll((long long)near) - 1 : lane;
			const uint32_t kj = (uint32_t)__shfl((int)kv, j);
			const bool eq = has && kj == kv;
			nbfar = nbfar || (has && !eq && kj - kv + (uint32_t)(2 * tol) <= (uint32_t)(4 * tol));
			eqm |= eq ? 1ull << j : 0ull;
			near &= near - 1ull;   // (0 stays 0)
		}
		// same = the chunk's candidates of this lane's row: the table again, by row
		wsync();
		if (lane < 32) L->btab[lane] = 0ull;
		wsync();
		if (act) atomicOr(&L->btab[r0], 1ull << lane);
		wsync();
		const unsigned long long same = act ? L->btab[r0] : 0ull;
		// a B group settles when all of it are B candidates with distinct kP1 (non-decreasing in
		// chunk order: compare with the previous member) and nothing else is within 2*tol
		const unsigned long long below = eqm & ((1ull << lane) - 1ull);
		const int prev = below ? 63 - __clzll((long long)below) : lane;
		const int kprev = __shfl(kP1, prev);
		const unsigned long long dupm = ballot(act && below != 0ull && kprev == kP1);
		const bool isB = bcand && !nbfar && (eqm & ~ballot(bcand)) == 0ull && (eqm & dupm) == 0ull;
		const unsigned long long grp = eqm;
		// A: no slot within the tolerance and nothing else within 2*tol but candidates of the same kv
		// with distinct kP1 -- in order, the first opens a slot and the rest vote on it exactly, so
		// the group settles as one new slot holding its whole fold (a lone candidate is the group
		// of one)
		const bool opener = act && nmatch == 0 && !nbfar && (eqm & dupm) == 0ull;
		// serial: matches batch mode cannot settle, crowded openers, B groups that did not qualify
		const bool dep1 = act && !isB && !opener;
		const unsigned long long bd = ballot(dep1);
		const unsigned long long le = lane == 63 ? ~0ull : ((1ull << (lane + 1)) - 1ull);
		// a group's first candidate after a serial candidate of its row would open its slot out of
		// order: it replays, and the rest of its group with it (they vote on its slot; their own
		// place in the row does not matter -- they open nothing)
		const bool lead = opener && below == 0ull;
		const bool depL = lead && (same & bd & le) != 0ull;
		const unsigned long long dlm = ballot(depL);
		const bool dep = dep1 || depL || (opener && (eqm & dlm) != 0ull);
#ifdef SVG_STAMPS
		{   // ballots with every lane active; the counts are wave-uniform
			const int w0 = __popcll(ballot(dep && nmatch >= 2)), w1 = __popcll(ballot(dep && nmatch == 1 && !bcand));
			const int w2 = __popcll(ballot(dep && bcand)), w3 = __popcll(ballot(dep && nmatch == 0));
			why[0] += w0; why[1] += w1; why[2] += w2; why[3] += w3;
		}
#endif
		// the group's first candidate opens the slot (rank among the row's openers); the group's
		// last one gives last and coverage end; all of its votes are in
		const int lastl = eqm ? 63 - __clzll((long long)eqm) : lane;
		const int kl = __shfl(kP1, lastl), ol = __shfl(off, lastl);
		const bool inr = lead && !dep && kv >= kp->low && kv <= high_b;
		const unsigned long long cm = ballot(inr);
		const int rank = __popcll(same & cm & (le >> 1));
		const bool mk = inr && n0 + rank < SPACE;
		if (lane < 32) L->rnew[lane] = 0xff;
		wsync();
		int nv = 0;
		if (mk) {
			nv = __popcll(eqm);
			L->pm[(int)r0 * PSTR + n0 + rank] =
				make_uint2(kv, m_pack_u(nv, kl, 0, gap_x(ol, kp->ix.gap), kP1, gap_x(off, kp->ix.gap)));   // no cold state
		}
		if (isB && (grp & ~le) == 0ull) {   // the group's last vote: votes += group size, last = its kP1
			nv = m_votes(tM) + __popcll(grp);
			L->pm[tslot].y = m_pack_u(nv, kP1, m_shift(tM), gap_x(off, kp->ix.gap), m_first(tM), m_fx(tM));
		}
		if (inr && (same & cm & ~le) == 0ull) L->rnew[r0] = (uint8_t)(n0 + rank + 1 < SPACE ? n0 + rank + 1 : SPACE);
		wsync();
		if ((lane >> 5) == E && (lane & 31) < ROWS) {
			const int v = L->rnew[lane & 31];
			if (v != 0xff) items_v = v;
		}
		for (int o = 32; o; o >>= 1) { const int t = __shfl_xor(nv, o); nv = t > nv ? t : nv; }
		nv = __builtin_amdgcn_readfirstlane(nv);
		if (max_vote[E] < nv) max_vote[E] = nv;
		wsync();
		return ballot(dep);
	}

	// ---------------------------------------------------------------- phases G+V for one (strand, end, round)
	template <int E>
	__device__ void replay(int s, int round)
	{
		const int lane = lane_id();
		const int np = rc.np[E];
		const int gap = kp->ix.gap;
		const uint32_t high_b = kp->high - (uint32_t)rc.rl[E];
		// candidate prefix over probes (probe order = subread_no, xk1)
		uint32_t total = 0;
		for (int p0 = 0; p0 < np; p0 += 64) {
			int p = p0 + lane;
			uint32_t h = p < np ? (uint32_t)L->pfwd[E][s][p] + L->pbwd[E][s][p] : 0u;
			uint32_t inc = wave_incl_scan(h);
			if (p < np) L->pcum[p + 1] = total + inc;
			total += __shfl(inc, 63);
		}
		if (lane == 0) L->pcum[0] = 0;
		wsync();
		STAMP(2);
		// gather in visiting order (probe p, then mid..last, then mid-1..first), lane c = candidate
		// c0 + c of the chunk; the next chunk's hit values are loaded while this one is voted
		auto locate_cand = [&](uint32_t cc, uint32_t &item, int &off, int &kP1) __attribute__((always_inline)) -> bool {
			int lo = 0, hi = np - 1;   // probe p with pcum[p] <= cc < pcum[p+1]
			while (lo < hi) { int m = (lo + hi + 1) >> 1; if (L->pcum[m] <= cc) lo = m; else hi = m - 1; }
			const int p = lo;
			const uint32_t j = cc - L->pcum[p];
			const uint32_t fwd = L->pfwd[E][s][p];
			const uint32_t mid = L->pmid[E][s][p];
			item = j < fwd ? mid + j : mid - 1 - (j - fwd);
			off = probe_off(E, p);
			kP1 = (gap == 1 ? p : p / gap) + 1;
			return false;
		};
		uint32_t nitem = 0, nval = 0;
		int noff = 0, nkp1 = 0;
		if ((uint32_t)lane < total) {
			const bool inl = locate_cand((uint32_t)lane, nitem, noff, nkp1);
			const uint32_t v = kp->ix.vals[inl ? 0u : nitem];
			nval = inl ? nitem : v;
		}
		for (uint32_t c0 = 0; c0 < total; c0 += CAND_CAP) {
			const uint32_t cn = total - c0 < CAND_CAP ? total - c0 : CAND_CAP;
			const uint32_t kv = nval - (uint32_t)noff;
			const int kvv = (int)kv, kov = (int)cand_pack(kv, nkp1, noff);
			if (c0 + CAND_CAP + (uint32_t)lane < total) {
				const bool inl = locate_cand(c0 + CAND_CAP + (uint32_t)lane, nitem, noff, nkp1);
				const uint32_t v = kp->ix.vals[inl ? 0u : nitem];
				nval = inl ? nitem : v;
			}
			STAMP(2);
			{
				const int m = (int)cn;
				unsigned long long serial = m == 64 ? ~0ull : ((1ull << m) - 1ull);
				if (round == 0 && kp->ii_end == 5 && m >= 8) serial = batch_create<E>(kvv, kov, m, high_b);
				if constexpr (!SJ) STAMP(6);   // diagnostics: batch mode (align variants; SJ uses 6 for junctions)
				if (kp->stats && lane == 0) {   // diagnostics: straight to the counters (no register kept live)
					atomicAdd(&kp->stats[26], (unsigned long long)(m - __popcll(serial)));
					atomicAdd(&kp->stats[27], (unsigned long long)__popcll(serial));
				}
				while (serial) {
					const int j = __ffsll((long long)serial) - 1;
					serial &= serial - 1ull;
					uint32_t kv = (uint32_t)rd(kvv, j);
					uint32_t pk = (uint32_t)rd(kov, j);
					vote_one<E>(kv, pk, round, high_b);
				}
			}
			wsync();
			STAMP(3);
		}
	}

	// ---------------------------------------------------------------- record helpers
	__device__ __forceinline__ void rec_zero(uint32_t *r) { if (lane_id() < 17) r[lane_id()] = 0; }

	// ---------------------------------------------------------------- table entries for top-K
	// An entry handle h is a table slot, or for PE end 0 an index into the compacted list.
	__device__ __forceinline__ bool compact(int e) const { return ENDS == 2 && e == 0; }
	__device__ __forceinline__ void ent_h(int e, int h, uint32_t &P, uint32_t &M, int &slot) const
	{
		if (compact(e)) {
			if (h < L->CAPL) { uint2 v = L->cl[h]; P = v.x; M = v.y; slot = L->cls[h]; }
			else { const uint32_t *o = ovf + 4 * h; P = o[0]; M = o[1]; slot = (int)o[2]; }
		} else {
			uint2 v = L->pm[h]; P = v.x; M = v.y; slot = h;
		}
	}
	// flattened used-slot index f (< U) -> handle; all lanes active (slot_of shuffles)
	__device__ __forceinline__ int handle_of(int e, int rs_v, int f) const
	{
		if (compact(e)) return f;
		return slot_of(e, rs_v, f);
	}

	// PE: end 0's used slots, in flattened row order, to the compact list (all lanes active)
	__device__ __forceinline__ void compact_end0()
	{
		const int lane = lane_id();
		int mine = lane < ROWS ? items_v : 0;
		int v = mine;
		for (int o = 1; o < 32; o <<= 1) { int t = __shfl_up(v, o); if ((lane & 31) >= o) v += t; }
		const int U = rd(v, ROWS - 1);
		for (int f0 = 0; f0 < U; f0 += 64) {
			int f = f0 + lane;
			int sl = slot_of(0, v, f);
			if (f < U) {
				uint2 pmv = L->pm[sl];
				if (f < L->CAPL) { L->cl[f] = pmv; L->cls[f] = (uint16_t)sl; }
				else { uint32_t *o = ovf + 4 * f; o[0] = pmv.x; o[1] = pmv.y; o[2] = (uint32_t)sl; }
			}
		}
		wsync();
	}

	// copy_vote_to_alignment_res (core-junction.c:1058-1071) for slot -> record r (pre-zeroed)
	__device__ void copy_vote(int e, int h, uint32_t *r)
	{
		const int lane = lane_id();
		uint32_t P, M;
		int slot;
		ent_h(e, h, P, M, slot);
		// indel_recorder_copy (sorted-hashtable.c:1144): triples while rec[3t] != 0 and 3t < 19
		int v = 0;
		if (lane < REC_LEN) v = slot_rec(e, slot, M, lane);
		const uint32_t cw = slot_cw(e, slot, M);
		unsigned long long z = ballot(lane < 19 && (lane % 3) == 0 && v == 0);
		int T = z ? (__ffsll((long long)z) - 1) / 3 : 7;   // number of triples copied
		int nrec = 3 * T;
		int last_ind = __shfl(v, nrec > 0 ? nrec - 1 : 0);
		int16_t rv = lane < nrec ? (int16_t)v : (int16_t)0;
		int16_t rv_hi = __shfl(rv, (2 * lane + 1) & 63);
		int16_t rv_lo = __shfl(rv, (2 * lane) & 63);
		if (lane < 11) r[MR_REC / 4 + lane] = (uint32_t)(uint16_t)rv_lo | ((uint32_t)(uint16_t)rv_hi << 16);
		if (lane == 0) {
			r[0] = P;
			r[2] = (uint32_t)(uint16_t)m_votes(M) | ((uint32_t)(uint16_t)end_sel(rc.applied, e) << 16);
			r[3] = (uint32_t)(uint8_t)(int8_t)(nrec > 0 ? last_ind : 0) << 8;   // noninf 0, indels
			r[15] = cw;      // confident_coverage_start | confident_coverage_end << 16
			r[16] = 0;
		}
	}

	// locate_gene_position_max(..., NULL, NULL, rl = 0), gene-algorithms.c:441-511
	__device__ int locate(uint32_t linear, int *chr, int *pos) const
	{
		const uint32_t *ce = kp->ix.chr_end;
		int ntot = (int)kp->ix.n_chr, lo = 0, hi = ntot, n;
		*chr = -1; *pos = -1;
		for (;;) {
			if (hi <= lo + 1) { n = lo - 2 > 0 ? lo - 2 : 0; break; }
			int mid = (lo + hi) / 2;
			if (ce[mid] > linear) hi = mid; else lo = mid + 1;
		}
		for (; n < ntot; n++) {
			if (ce[n] > linear) {
				*pos = n == 0 ? (int)linear : (int)(linear - ce[n - 1]);
				if (linear > ce[n] + 15u - (uint32_t)kp->ix.padding) return 1;
				if (*pos < kp->ix.padding) return 1;
				*pos -= kp->ix.padding;
				*chr = n;
				return 0;
			}
		}
		return -1;
	}

	// ---------------------------------------------------------------- subjunc helpers (SJ variant)
	// gvindex_get (gene-value-index.c:1118-1136 via gvindex_get_string): 'N' past the array
	// .array bytes of the current donor search are staged in two 64-byte LDS windows
	// (left / right half of the junction); a byte outside them is read from HBM
	__device__ __forceinline__ int vbyte(int w, uint32_t byte) const
	{
		const uint32_t d = byte - wb[w];
		return d < 64 ? (int)L->gwin[w][d] : (int)kp->ix.values[byte];
	}
	__device__ __forceinline__ char gv_get(int w, uint32_t pos) const
	{
		const DevIndex &ix = kp->ix;
		uint32_t byte = (pos - ix.start_base_offset) >> 2, bit = pos % 4 * 2;
		if (byte >= ix.values_bytes - 1) return 'N';
		return "AGCT"[(vbyte(w, byte) >> bit) & 3];
	}
	// stage the window of side w starting at array position pos0 (all lanes)
	__device__ void load_window(int w, uint32_t pos0)
	{
		const DevIndex &ix = kp->ix;
		wb[w] = (pos0 - ix.start_base_offset) >> 2;
		const uint32_t idx = wb[w] + (uint32_t)lane_id();
		L->gwin[w][lane_id()] = idx < ix.values_bytes ? ix.values[idx] : 0;
	}

	// match_chro (gene-value-index.c:856-959, space_type = base): matched bases of
	// read[0..len) against the array at pos; 0 whenever the walk reaches the array end
	__device__ int match_chro(int w, const char *read, int read_len, int at, uint32_t pos, int len) const
	{
		const DevIndex &ix = kp->ix;
		if ((uint32_t)(pos + len) >= ix.length + ix.start_point) return 0;
		if (pos > 0xffff0000u) return 0;
		uint32_t byte = (pos - ix.start_base_offset) >> 2, bit = pos % 4 * 2;
		if (byte >= ix.values_bytes) return 0;
		if (byte + (bit / 2 + len) / 4 >= ix.values_bytes) return 0;   // the walk would hit the end
		int ret = 0;
		int iv = vbyte(w, byte);
		for (int i = 0; i < len; i++) {
			int tt = (iv >> bit) & 3;
			int q = at + i;
			char c = q < read_len ? read[q] : 0;   // the reference's read buffer is NUL-terminated
			ret += c == 'A' ? tt == 0 : c == 'G' ? tt == 1 : c == 'C' ? tt == 2 : c == 0 ? 0 : tt == 3;
			bit += 2;
			if (bit == 8) { byte++; iv = vbyte(w, byte); bit = 0; }
		}
		return ret;
	}

	__device__ static bool donor_pair(char a, char b)
	{
		return (a == 'G' && b == 'T') || (a == 'A' && b == 'G') || (a == 'A' && b == 'C') || (a == 'C' && b == 'T');
	}

	// donor_score (core-junction.c:3675-3834; no fusion/long-del, max_insertion_at_junctions 0),
	// lanes = tested split points.  The reference keeps the first split point (in its
	// mid-outward visiting order) with the strictly best score, so the wave takes the
	// maximum score and, among equal scores, the lowest visiting index.  Returns
	// (1+best)/100 or 0 and the split point / GT-AG strand / found flag.
	__device__ int donor(int e, uint32_t left, uint32_t right, int lio, int normal, int gs, int ge, int *split, int *gtag, int *found)
	{
		const svg_params &p = kp->p;
		const int lane = lane_id();
		const char *read = L->text[e][cur_strand];
		const int rl = end_sel(rc.rl, e);
		const bool need_donor = p.check_donor_at_junctions != 0;
		const int allow = p.more_accurate_fusions ? 0 : 1;
		const int mid = (gs + ge) / 2, n = ge - gs;
		int best = -111111, bi = 0x7fffffff, bstrand = -1, bsp = -1;
		{
			// split points visited lie in [gs-1, ge+1] and pass only inside [17, rl-17]; the
			// windows cover 20 bases before the lowest to 17 after the highest
			int lo_sp = gs - 1 > JCW ? gs - 1 : JCW;
			uint32_t l0 = left + (uint32_t)(lo_sp + lio), r0 = right + (uint32_t)lo_sp;
			load_window(0, l0 >= 20u ? l0 - 20u : 0u);
			load_window(1, r0 >= 20u ? r0 - 20u : 0u);
			wsync();
		}
		int carry_dr1 = 0;   // dr[1] left by the last earlier split point that fetched it (normal branch)
		for (int i0 = 0; i0 < n; i0 += 64) {
			int i = i0 + lane;
			int sc = -0x7fffffff, sp = 0;
			bool cand = false, dr_set = false;
			char dl0 = 0, dl1 = 0, dr0 = 0, dr1 = 0;
			if (i < n) {
				sp = mid + ((i % 2) ? -((i + 1) / 2) : ((1 + i) / 2));
				if (sp <= rl - JCW && sp >= JCW) {
					bool ok = false;
					if (p.prefer_donor_receptor_junctions) {
						if (normal) {
							dl0 = gv_get(0, left + sp + lio); dl1 = gv_get(0, left + sp + lio + 1);
							if (donor_pair(dl0, dl1)) {
								dr0 = gv_get(1, right + sp - 2); dr1 = gv_get(1, right + sp - 1);
								dr_set = true;
								if (donor_pair(dr0, dr1))
									ok = ((dl0 == 'G' && dl1 == 'T' && dr0 == 'A' && dr1 == 'G') || (dl0 == 'C' && dl1 == 'T' && dr0 == 'A' && dr1 == 'C'))
									     && ((dl0 == 'C' && dl1 == 'T') || (dl0 == 'G' && dl1 == 'T'));
							}
						} else {
							dl0 = gv_get(1, right + sp + lio); dl1 = gv_get(1, right + sp + lio + 1);
							dr0 = gv_get(0, left + sp - 2); dr1 = gv_get(0, left + sp - 1);
							dr_set = true;
							ok = donor_pair(dl0, dl1) && donor_pair(dr0, dr1)
							     && ((dl0 == 'G' && dl1 == 'T' && dr0 == 'A' && dr1 == 'G') || (dl0 == 'C' && dl1 == 'T' && dr0 == 'A' && dr1 == 'C'))
							     && ((dl0 == 'C' && dl1 == 'T') || (dl0 == 'G' && dl1 == 'T'));
						}
					}
					if (ok || !need_donor) {
						int lm, rm, ln, rn;
						if (normal) {
							lm = match_chro(0, read, rl, sp - JCW, left + sp - JCW + lio, JCW);
							if (lm > JCW - 2) {
								rm = match_chro(1, read, rl, sp, right + sp, JCW);
								if (rm >= 2 * JCW - lm - allow) {
									ln = match_chro(0, read, rl, sp, left + sp + lio, JCW);
									rn = match_chro(1, read, rl, sp - JCW, right + sp - JCW, JCW);
									if (ln <= JCW - 5 && rn <= JCW - 5) { sc = 100 * ((ok ? 3000 : 0) + lm + rm - ln - rn); cand = true; }
								}
							}
						} else {
							rm = match_chro(1, read, rl, sp - JCW, right + sp - JCW, JCW);
							lm = match_chro(0, read, rl, sp, left + sp + lio, JCW);
							rn = match_chro(1, read, rl, sp, right + sp, JCW);
							ln = match_chro(0, read, rl, sp - JCW, left + lio + sp - JCW, JCW);
							if (lm + rm >= 2 * JCW - allow && ln <= JCW - 5 && rn <= JCW - 5) { sc = 100 * ((ok ? 3000 : 0) + lm + rm - ln - rn); cand = true; }
						}
					}
				}
			}
			// the strand test uses the dr[] the reference's loop holds at that point: this split
			// point's when fetched, else the last earlier fetch (only reachable without the donor test)
			unsigned long long dm = ballot(dr_set);
			unsigned long long below = dm & ((1ull << lane) - 1ull);
			int prev_dr1 = below ? __shfl((int)dr1, 63 - __clzll(below)) : carry_dr1;
			int use_dr1 = dr_set ? (int)dr1 : prev_dr1;
			if (dm) carry_dr1 = __shfl((int)dr1, 63 - __clzll(dm));
			int strand = (dl0 == 'G' || use_dr1 == 'G') ? 1 : 0;
			int cmax = wave_max(cand ? sc : -0x7fffffff);
			unsigned long long wm = ballot(cand && sc == cmax);
			if (wm && cmax > best) {
				int w = __ffsll((long long)wm) - 1;   // lowest visiting index in this chunk
				best = cmax;
				bi = i0 + w;
				bsp = __shfl(sp, w);
				bstrand = __shfl(strand, w);
			}
		}
		(void)bi;
		if (best > 0) {
			*split = bsp; *found = best >= 290000; *gtag = bstrand;
			return (1 + best) / 100;
		}
		return 0;
	}

	// junction part of copy_vote_to_alignment_res (core-junction.c:1073-1334, no fusion):
	// every other used slot of the table is a minor-half candidate.  The J-independent
	// filters run lane-parallel; the is_better chain and donor scoring run in slot order.
	__device__ void junction(int e, int mh, uint32_t *r, uint32_t *J, int rs_v, int U)
	{
		const svg_params &p = kp->p;
		const int lane = lane_id();
		uint32_t Mpos, MM;
		int ms;
		ent_h(e, mh, Mpos, MM, ms);
		const int Mv = m_votes(MM);
		const uint32_t mw = slot_cw(e, ms, MM);
		const int Mcs = (int)(mw & 0xffff), Mce = (int)(mw >> 16);
		const int rl = end_sel(rc.rl, e);
		int Jv = 0, Jcs = 0, Jce = 0, Jsplit = 0, Jnormal = 0, Jdio = 0;
		// long reads (core-junction.c, curr_read_len > EXON_LONG_READ_LENGTH): the indel offsets
		// accumulated over each half's indel recorder shift the smaller half's donor tests
		int major_ind = 0;
		if (rl > 160 && m_spilled(MM)) {   // an unspilled recorder is (first, last, 0): offset 0
			const uint32_t *mcs = cold_slot(end_sel(cold, e), ms);
			for (int kx = 0; kx < SVG_MAX_INDEL_SECTIONS; kx++) {
				if (!cold_rec(mcs, kx * 3)) break;
				major_ind += cold_rec(mcs, kx * 3 + 2);
			}
		}
		uint32_t Jpos = 0;
		int flags = (int)(r[1] & 0xffff);
		bool upd = false;
		for (int f0 = 0; f0 < U; f0 += 64) {
			int f = f0 + lane;
			int hh = handle_of(e, rs_v, f);   // all lanes active
			bool ok = f < U && hh != mh;
			uint32_t P = 0, MMv = 0;
			int V = 0, cs = 0, ce = 0;
			int sl = 0;
			long long dist = 0;
			if (ok) {
				ent_h(e, hh, P, MMv, sl);
				V = m_votes(MMv);
				dist = (long long)Mpos - (long long)P;
				ok = Mv >= V && (dist < 0 ? -dist : dist) <= (long long)p.maximum_intron_length;
			}
			// the coverage (cold state, HBM) only for slots within intron distance -- usually none
			if (!ballot(ok)) continue;
			if (ok) {
				uint32_t w = slot_cw(e, sl, MMv);
				cs = (int)(w & 0xffff); ce = (int)(w >> 16);
				ok = cs != Mcs && ce != Mce;
				if (ok) ok = (Mcs > cs) ? (Mpos >= P) : (Mpos <= P);   // test_junction_minor
				if (ok) {
					int ov = (Mcs > cs) ? ce - Mcs : Mce - cs;
					ok = ov <= 14 && abs((int)dist) >= 6;
				}
			}
			unsigned long long m = ballot(ok);
			while (m) {
				int b = __ffsll((long long)m) - 1;
				m &= m - 1;
				uint32_t Pb = (uint32_t)rd((int)P, b);
				int Vb = rd(V, b), csb = rd(cs, b), ceb = rd(ce, b);
				// is_better_inner, core-junction.c:961
				int old_intron = (int)abs32u(Mpos - Jpos), intron = (int)abs32u(Mpos - Pb);
				int cl = ceb - csb, jl = Jce - Jcs;
				bool better = Vb > Jv || (Vb == Jv && cl > jl) || (Vb == Jv && cl == jl && intron < old_intron);
				if (!better) continue;
				int gs = (Mcs > csb) ? ceb - 8 : Mce - 8;
				int ge = (Mcs < csb) ? csb + 8 : Mcs + 8;
				int normal = 1 != (int)(Mcs > csb) + (int)(Mpos > Pb);
				int split = 0, gtag = 0, found = 0;
				int minor_ind = 0, lio = 0;
				if (rl > 160) {
					const uint32_t Mb = (uint32_t)rd((int)MMv, b);
					const uint32_t *ncs = cold_slot(end_sel(cold, e), rd(sl, b));
					for (int kx = 0; kx < SVG_MAX_INDEL_SECTIONS && m_spilled(Mb); kx++) {
						if (!cold_rec(ncs, kx * 3)) break;
						minor_ind += cold_rec(ncs, kx * 3 + 2);
					}
					lio = Mpos < Pb ? major_ind : minor_ind;   // the larger half's offset is 0
				}
				int sc = donor(e, Mpos < Pb ? Mpos : Pb, Mpos > Pb ? Mpos : Pb, lio, normal, gs > 0 ? gs : 0, ge < rl ? ge : rl,
				               &split, &gtag, &found);
				if (sc > 0) {
					Jpos = Pb; Jv = Vb; Jcs = csb; Jce = ceb; Jsplit = split; Jnormal = normal;
					Jdio = (minor_ind & 0xf) | ((major_ind & 0xf) << 4);   // double_indel_offset
					flags &= ~0x3;
					if (!found || gtag > 2) flags |= 3;
					else flags = gtag ? (flags | 1) : (flags & ~1);
					flags &= ~4;
					upd = true;
				}
			}
		}
		if (upd && lane == 0) {
			// subjunc_result_t: split_point, minor_votes | double_indel_offset 0, indel_at_junction 0,
			// small/large_side_increasing_coordinate = !normal / normal of the last update
			J[0] = (uint32_t)(uint16_t)Jsplit | ((uint32_t)(uint16_t)Jv << 16);
			J[1] = (uint32_t)(uint8_t)Jdio | ((uint32_t)(Jnormal ? 0 : 1) << 16) | ((uint32_t)(Jnormal ? 1 : 0) << 24);
			J[2] = Jpos;
			J[3] = (uint32_t)(uint16_t)Jcs | ((uint32_t)(uint16_t)Jce << 16);
			r[1] = (r[1] & 0xffff0000u) | (uint32_t)(uint16_t)flags;
		}
		wsync();
	}

	// flattened (row-major) used-slot index f -> slot, given the inclusive row prefix rs_v
	// (lane 32*e+r holds items[0..r] of table e).  Must run with every lane active: the
	// cross-lane read (ds_bpermute) returns nothing useful from inactive source lanes.
	__device__ __forceinline__ int slot_of(int e, int rs_v, int f) const
	{
		int row = 0;
#pragma unroll
		for (int r = 0; r < ROWS - 1; r++) row += (rd(rs_v, e * 32 + r) <= f);
		int start = __shfl(rs_v, (e * 32 + row - 1) & 63);
		if (row == 0) start = 0;
		return row * PSTR + (f - start);
	}

	// ---------------------------------------------------------------- phase K
	__device__ __forceinline__ void topk(int strand)
	{
		const svg_params &p = kp->p;
		const int lane = lane_id();
		int top[2][3] = {{0, 0, 0}, {0, 0, 0}};
		int nsimp[2] = {0, 0};
		constexpr int TS = 3;   // p.top_scores, validated == 3 on the host
		// inclusive row prefix of used slots per table
		int mine = ((lane & 31) < ROWS) ? items_v : 0;
		int rs_v = 0;
		{
			int lo = lane & 31;
			int v = mine;
			for (int o = 1; o < 32; o <<= 1) { int t = __shfl_up(v, o); if (lo >= o) v += t; }
			rs_v = v;
		}
		int U[2];
		U[0] = rd(rs_v, ROWS - 1);
		U[1] = ENDS == 2 ? rd(rs_v, 32 + ROWS - 1) : 0;
		// handle of flattened index f = lane (first 64 used slots), computed once per table
		int sl0[2];
		sl0[0] = handle_of(0, rs_v, lane);
		sl0[1] = ENDS == 2 ? handle_of(1, rs_v, lane) : 0;
		// single end: the handles of used slots 64..255 too, computed once for the six passes below
		// (slot_of is 29 readlanes; a heavy read's table holds 100-260 used slots)
		int slh[ENDS == 1 ? 3 : 1];
		if constexpr (ENDS == 1) {
#pragma unroll
			for (int c = 0; c < 3; c++) slh[c] = U[0] > 64 * (c + 1) ? handle_of(0, rs_v, 64 * (c + 1) + lane) : 0;
		}
		auto hcache = [&](int e, int f0, int f) __attribute__((always_inline)) -> int {
			if (f0 == 0) return e ? sl0[1] : sl0[0];
			if constexpr (ENDS == 1) {
				if (f0 <= 192) return f0 == 64 ? slh[0] : (f0 == 128 ? slh[1] : slh[2]);
			}
			return handle_of(e, rs_v, f);   // all lanes active
		};
		for (int e = 0; e < ENDS; e++) {
			// top-3 distinct over table votes and stored results (update_top_three, core-junction.c:908-922):
			// one scan -- each lane keeps the three largest distinct votes of its slots, then three wave
			// maxima, each taking its value off the lanes that hold it (a heavy read's table has 100-260
			// slots: one pass over them instead of one per rank)
			int a = 0, b = 0, c = 0;
			// (branch-free: one max / min bubble step per place -- the if-chain was lowered to a
			// dynamically indexed private array, i.e. scratch)
#define TOP3_INS(v_) do { const int v = (v_); \
				if (v > c && v != a && v != b) { \
					const int t1 = a < v ? a : v, t2 = b < t1 ? b : t1; \
					a = a > v ? a : v; b = b > t1 ? b : t1; c = c > t2 ? c : t2; } } while (0)
			for (int f0 = 0; f0 < U[e]; f0 += 64) {
				int f = f0 + lane;
				int sl = hcache(e, f0, f);
				if (f < U[e]) {
					uint32_t P, M;
					int cs_;
					ent_h(e, sl, P, M, cs_);
					TOP3_INS(m_votes(M));
				}
			}
			if (lane < p.multi_best) TOP3_INS(rec_votes(L->res[e][lane]));
#undef TOP3_INS
			for (int t = 0; t < TS; t++) {
				const int best = wave_max(a);
				top[e][t] = best;
				if (a == best) { a = b; b = c; c = 0; }
			}
		}
		STAMP(8);
		// candidate lists (simples)
		for (int e = 0; e < ENDS; e++) {
			int ns = 0;
			for (int t = 0; t < TS; t++) {
				int N = top[e][t];
				if (ns >= p.max_vote_simples) break;
				if (N < 1 || (top[e][0] - N > p.max_vote_number_cutoff)) break;
				for (int f0 = 0; f0 < U[e] && ns < p.max_vote_simples; f0 += 64) {
					int f = f0 + lane;
					int hd = hcache(e, f0, f), v = -1;
					uint32_t P = 0, M = 0;
					int slot = 0;
					if (f < U[e]) { ent_h(e, hd, P, M, slot); v = m_votes(M); }
					bool sel = f < U[e] && v == N && v >= p.min_votes_second;
					unsigned long long sm = ballot(sel);
					int at = ns + lanes_below(sm);
					if constexpr (SJ) {
						// insert_big_margin_record (core-junction.c:2276-2277,789) for every slot the
						// reference's scan visits before max_vote_simples is reached, first value only
						if (t == 0 && p.do_big_margin_filtering_for_junctions) {
							STAMP(4);
							const bool elig = f < U[e] && at < p.max_vote_simples && v >= top[e][TS - 1];
							if (ballot(elig)) {
								const uint32_t cw = elig ? slot_cw(e, slot, M) : 0u;
								big_margin_merge(e, elig, v, cw);
							}
							STAMP(7);
						}
					}
					if (sel && at < p.max_vote_simples) {
						L->simp_pos[e][at] = P;
						L->simp_slot[e][at] = (uint16_t)hd;
						L->simp_votes[e][at] = (uint16_t)v;
					}
					ns += __popcll(sm);
					if (ns > p.max_vote_simples) ns = p.max_vote_simples;
				}
				for (int i = 0; i < p.multi_best; i++) {
					if (ns >= p.max_vote_simples) break;
					if (rec_votes(L->res[e][i]) == N) {
						if (lane == 0) {
							L->simp_pos[e][ns] = rec_pos(L->res[e][i]);
							L->simp_slot[e][ns] = (uint16_t)(0x8000 | i);
							L->simp_votes[e][ns] = (uint16_t)N;
						}
						ns++;
					}
				}
			}
			nsimp[e] = ns;
		}
		wsync();
		for (int e = 0; e < ENDS; e++) {
			for (int i = 0; i < 3; i++) rec_zero(L->tmp[e][i]);
			if constexpr (SJ) { if (lane < 12) L->jtmp[e][lane / 4][lane % 4] = 0; }
		}
		wsync();
		STAMP(9);
		int cur[2] = {0, 0};
		int ncomb = 0;
		if (ENDS == 2) {
			// all valid pairs, keep the first 3 by (score desc, pair order asc)
			int n0 = nsimp[0], n1 = nsimp[1];
			int npairs = n0 * n1;
			// each simple located once (up to 64 x 64 pairs would locate both ends of every pair)
			for (int e = 0; e < 2; e++) {
				if (lane < nsimp[e]) {
					int c, q;
					const int err = locate(L->simp_pos[e][lane], &c, &q);
					L->simp_loc[e & (ENDS - 1)][lane] = q;
					L->simp_chr[e & (ENDS - 1)][lane] = (int16_t)(err == 0 ? c : -1);
				}
			}
			wsync();
			// each lane keeps its own first 3 pairs by (score desc, pair order asc) -- its pairs come
			// in ascending order -- and the wave's first 3 are then taken from the lanes' heads
			int ls0 = -1, ls1 = -1, ls2 = -1, li0 = 0x7fffffff, li1 = 0x7fffffff, li2 = 0x7fffffff;
			for (int q0 = 0; q0 < npairs; q0 += 64) {
				int q = q0 + lane;
				int sc = -1;
				if (q < npairs) {
					int i = q / n1, j = q - i * n1;
					int va = L->simp_votes[0][i], vb = L->simp_votes[1][j];
					int mx = va > vb ? va : vb, mn = va < vb ? va : vb;
					if (mx >= p.min_votes_first) {
						int pe = 0, same = 0;
						const int c1 = L->simp_chr[0][i], c2 = L->simp_chr[ENDS - 1][j];
						const int q1 = L->simp_loc[0][i], q2 = L->simp_loc[ENDS - 1][j];
						if (c1 >= 0 && c2 >= 0) {
							long long tlen = (long long)q1 - q2;
							tlen = abs((int)tlen);
							tlen += (q1 > q2) ? rc.rl[0] : rc.rl[1];
							uint32_t tli = (uint32_t)tlen;
							if (c1 == c2) {
								same = 1;
								if (tli >= (uint32_t)p.min_pair_distance && tli <= (uint32_t)p.max_pair_distance) pe = 1;
							}
						}
						if (pe || mn >= p.min_votes_first) sc = (va + vb) * (pe ? 1300 : (same ? 1000 : 800));
					}
				}
				// (an equal score keeps the earlier pair ahead: insert after the entries >= sc)
				if (sc > ls2) {
					if (sc > ls0) { ls2 = ls1; li2 = li1; ls1 = ls0; li1 = li0; ls0 = sc; li0 = q; }
					else if (sc > ls1) { ls2 = ls1; li2 = li1; ls1 = sc; li1 = q; }
					else { ls2 = sc; li2 = q; }
				}
			}
			// the wave's first three pairs as scalars (no arrays: a dynamically indexed one lives in scratch)
			int s0 = -1, s1 = -1, s2 = -1, q0 = 0, q1 = 0, q2 = 0, nfound = 0;
#pragma unroll
			for (int r = 0; r < 3; r++) {
				const int m = wave_max(ls0);
				if (m < 0) break;
				const int qi = wave_min(ls0 == m ? li0 : 0x7fffffff);
				if (r == 0) { s0 = m; q0 = qi; } else if (r == 1) { s1 = m; q1 = qi; } else { s2 = m; q2 = qi; }
				nfound++;
				if (li0 == qi) { ls0 = ls1; li0 = li1; ls1 = ls2; li1 = li2; ls2 = -1; li2 = 0x7fffffff; }
			}
			ncomb = nfound < p.max_vote_combinations ? nfound : (p.max_vote_combinations > 0 ? p.max_vote_combinations : 0);
			// merge_sort -> selection sort ascending by score (core.c:4716-4729), unstable: position 0
			// takes the first strictly smaller of positions 1, 2, then position 1 the smaller of 1, 2
			{
				int mj = 0, sm = s0;
				if (ncomb > 1 && sm - s1 > 0) { mj = 1; sm = s1; }
				if (ncomb > 2 && sm - s2 > 0) mj = 2;
				if (mj == 1) { int t = s0; s0 = s1; s1 = t; t = q0; q0 = q1; q1 = t; }
				else if (mj == 2) { int t = s0; s0 = s2; s2 = t; t = q0; q0 = q2; q2 = t; }
				if (ncomb > 2 && s1 - s2 > 0) { int t = s1; s1 = s2; s2 = t; t = q1; q1 = q2; q2 = t; }
			}
			if (ncomb > 0) {
				for (int e = 0; e < 2; e++) {
					for (int i = ncomb - 1; i >= 0; i--) {
						if (cur[e] >= p.multi_best) break;
						const int qq = i == 0 ? q0 : (i == 1 ? q1 : q2);
						const int si = e ? qq % n1 : qq / n1;
						uint32_t ps = L->simp_pos[e][si];
						bool ex = false;
						for (int j = 0; j < cur[e]; j++) if (rec_pos(L->tmp[e][j]) == ps) ex = true;
						if (ex) continue;
						emit(e, si, cur[e], rs_v, U[e]);
						cur[e]++;
					}
				}
			}
		}
		STAMP(10);
		if (ncomb == 0) {
			if (nsimp[0] == 0 && lane == 0) rec_set_noninf(L->res[0][0], 0);
			if (ENDS == 2 && nsimp[ENDS - 1] == 0 && lane == 0) rec_set_noninf(L->res[ENDS - 1][0], 0);
			wsync();
			for (int e = 0; e < ENDS; e++)
				for (int i = 0; i < nsimp[e]; i++) {
					if (cur[e] >= p.multi_best) break;
					if ((int)L->simp_votes[e][i] < p.min_votes_first) continue;
					uint32_t ps = L->simp_pos[e][i];
					bool ex = false;
					for (int j = 0; j < cur[e]; j++) if (rec_pos(L->tmp[e][j]) == ps) ex = true;
					if (ex) continue;
					emit(e, i, cur[e], rs_v, U[e]);
					cur[e]++;
				}
		}
		wsync();
		for (int e = 0; e < ENDS; e++)
			for (int i = 0; i < p.multi_best; i++) {
				if (i < cur[e]) { if (lane < 17) L->res[e][i][lane] = L->tmp[e][i][lane]; }
				else if (lane == 0) rec_set_votes(L->res[e][i], 0);
				if constexpr (SJ) {
					if (p.do_breakpoint_detection) {
						if (i < cur[e]) { if (lane < 4) L->jres[e][i][lane] = L->jtmp[e][i][lane]; }
						else if (lane == 0) L->jres[e][i][0] &= 0xffffu;   // minor_votes = 0
					}
				}
			}
		wsync();
	}

	// write simple si of end e as tmp record slot c
	__device__ __forceinline__ void emit(int e, int si, int c, int rs_v, int U)
	{
		int sl = L->simp_slot[e][si];
		if (sl & 0x8000) {
			if (lane_id() < 17) L->tmp[e][c][lane_id()] = L->res[e][sl & 3][lane_id()];
			if constexpr (SJ) { if (lane_id() < 4) L->jtmp[e][c][lane_id()] = L->jres[e][sl & 3][lane_id()]; }
		} else {
			copy_vote(e, sl, L->tmp[e][c]);
			// result_flags: IS_NEGATIVE_STRAND mask of the slot (every slot of a table has the table's strand)
			if (lane_id() == 0) L->tmp[e][c][1] = cur_strand ? (uint32_t)SVG_NEGATIVE_STRAND_FLAG : 0u;
			if constexpr (SJ) {
				if (kp->p.do_breakpoint_detection) {
					wsync();
					STAMP(4);
					junction(e, sl, L->tmp[e][c], L->jtmp[e][c], rs_v, U);
					STAMP(6);
				}
			}
		}
		wsync();
	}

	// insert_big_margin_record (core-junction.c:789-811) for every eligible lane of a chunk,
	// in lane order.  Each insertion puts the new record before the first one with votes
	// <= its own, so the record list is always the top size/3 of all insertions so far under
	// (votes desc, newer first) -- the chunk's top-3 by that key are merged with the list.
	__device__ void big_margin_merge(int e, bool elig, int votes, uint32_t cw)
	{
		const int size = kp->p.big_margin_record_size;   // 0..2 (no records) or 3, 6, 9
		if (size < 3) return;
		const int lane = lane_id(), ns = size / 3, rl = end_sel(rc.rl, e);
		const int rs = (int)(cw & 0xffff), re = (int)(cw >> 16);
		const uint32_t pay = cur_strand ? (uint32_t)(uint16_t)(rl - re) | ((uint32_t)(uint16_t)(rl - rs) << 16)
		                                : (uint32_t)(uint16_t)rs | ((uint32_t)(uint16_t)re << 16);
		int key = elig ? (((votes & 255) << 8) | (64 + lane)) : -1;
		int nk[3] = {-1, -1, -1};
		uint32_t np_[3] = {0, 0, 0};
		for (int t = 0; t < ns; t++) {
			const int m = wave_max(key);
			if (m < 0) break;
			const int l = (m & 255) - 64;
			nk[t] = m;
			np_[t] = (uint32_t)rd((int)pay, l);
			if (lane == l) key = -1;
		}
		if (lane == 0) {
			uint16_t *bm = L->bm[e];
			int ok[3];
			uint32_t op[3];
			for (int i = 0; i < ns; i++) { ok[i] = ((int)bm[3 * i] << 8) | (3 - i); op[i] = bm[3 * i + 1] | ((uint32_t)bm[3 * i + 2] << 16); }
			int rk[3];
			uint32_t rp[3];
			int a = 0, b = 0;
			for (int k = 0; k < ns; k++) {
				const bool takeN = a < ns && nk[a] >= 0 && (b >= ns || nk[a] > ok[b]);
				if (takeN) { rk[k] = nk[a] >> 8; rp[k] = np_[a]; a++; }
				else { rk[k] = ok[b] >> 8; rp[k] = op[b]; b++; }
			}
			for (int k = 0; k < ns; k++) {
				bm[3 * k] = (uint16_t)rk[k];
				bm[3 * k + 1] = (uint16_t)(rp[k] & 0xffff);
				bm[3 * k + 2] = (uint16_t)(rp[k] >> 16);
			}
		}
		wsync();
	}

	// voting of one end for one strand: init_gene_vote + subread loop + shift-indel round
	template <int E>
	__device__ __forceinline__ void vote_end(int strand)
	{
		nshift[E] = 0;
		if (rc.np[E] == 0) { table_reset<E>(); return; }
		for (int round = 0; round < 2; round++) {
			table_reset<E>();
			replay<E>(strand, round);
			if (nshift[E] == 0) break;
		}
	}

	// ---------------------------------------------------------------- one read
	// ---------------------------------------------------------------- read text
	// Aligned dwords covering [seq+o, seq+o+len) (never past the page holding the last
	// byte), WPL per lane; a read <= 256 bp is one load per lane (+1 on lane 0).
	static constexpr int WPL = (MAXL + 6) / 256 + 1;
	uint32_t tw[ENDS][WPL];
	int t_shift[ENDS], t_len[ENDS];

	__device__ __forceinline__ void prefetch_text(uint64_t r)
	{
		const int lane = lane_id();
		for (int e = 0; e < ENDS; e++) {
			int len = e ? kp->len2[r] : kp->len1[r];
			if (len > SVG_READ_KEEP) len = SVG_READ_KEEP;   // read_line keeps MAX_READ_LENGTH-1 (input-files.c:277)
			if (len > MAXL) {   // host-validated; never index LDS past the text buffer
				if (lane == 0) atomicOr(kp->err, 2u);
				len = 0;
			}
			t_len[e] = __builtin_amdgcn_readfirstlane(len);   // (uniform: the read's offsets / probe counts stay scalar)
			if constexpr (!SJ) continue;   // the vote step itself never reads the text
			const char *seq = e ? kp->seq2 : kp->seq1;
			const uint64_t o = e ? kp->off2[r] : kp->off1[r];
			uintptr_t a = (uintptr_t)(seq + o);
			const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
			t_shift[e] = (int)(a & 3);
			int nwd = (t_shift[e] + len + 3) >> 2;
#pragma unroll
			for (int k = 0; k < WPL; k++) {
				int i = lane + 64 * k;
				tw[e][k] = i < nwd ? w[i] : 0u;
			}
		}
	}

	// probe records of probe_kernel: RPL per lane (prefetched with the text when small)
	static constexpr int RPL = (ENDS * 2 * MAXP + 63) / 64;
	static constexpr bool PRE_RECS = RPL <= 2;
	uint2 trec[PRE_RECS ? RPL : 1];
	uint64_t t_r;

	__device__ __forceinline__ void prefetch_recs(uint64_t r)
	{
		t_r = r;
		if constexpr (PRE_RECS) {
			const int per = ENDS * 2 * kp->nps;
#pragma unroll
			for (int k = 0; k < RPL; k++) {
				int i = lane_id() + 64 * k;
				trec[k] = i < per ? rec_at(r, i) : make_uint2(0, 0);
			}
		}
	}

	__device__ __forceinline__ uint2 rec_at(uint64_t r, int i) const
	{
		const uint32_t sd = kp->prec_stride;
		return sd ? kp->precs[(uint64_t)i * sd + r] : kp->precs[r * (uint64_t)(ENDS * 2 * kp->nps) + i];
	}

	__device__ __forceinline__ void stage_probes()
	{
		const int nps = kp->nps, per = ENDS * 2 * nps;
#pragma unroll
		for (int k = 0; k < (PRE_RECS ? RPL : (ENDS * 2 * MAXP + 63) / 64); k++) {
			int i = lane_id() + 64 * k;
			if (i < per) {
				uint2 rec;
				if constexpr (PRE_RECS) rec = trec[k < RPL ? k : 0];
				else rec = rec_at(t_r, i);
				int e = i / (2 * nps), rem = i - e * 2 * nps, st = rem >= nps ? 1 : 0, q = rem - st * nps;
				L->pmid[e][st][q] = rec.x;
				L->pfwd[e][st][q] = (uint16_t)(rec.y & 0xffff);
				L->pbwd[e][st][q] = (uint16_t)(rec.y >> 16);
			}
		}
		wsync();
	}

	// prefetched words -> LDS staging (the vote table, free at this point) -> both strands
	__device__ __forceinline__ void stage_text()
	{
		const svg_params &p = kp->p;
		const int lane = lane_id();
		for (int e = 0; e < ENDS; e++) rc.rl[e] = t_len[e];
		if constexpr (!SJ) return;
		for (int e = 0; e < ENDS; e++) {
			uint32_t *stg = (uint32_t *)(L->pm + e * (NSLOT / 2));
#pragma unroll
			for (int k = 0; k < WPL; k++) stg[lane + 64 * k] = tw[e][k];
		}
		wsync();
		for (int e = 0; e < ENDS; e++) {
			const uint8_t *b = (const uint8_t *)(L->pm + e * (NSLOT / 2)) + t_shift[e];
			const int len = rc.rl[e], rev = e ? p.reverse_r2 : p.reverse_r1;
			for (int i = lane; i < len; i += 64) {
				char c = (char)b[i], c2 = (char)b[len - 1 - i];
				L->text[e][0][i] = rev ? comp(c2) : c;
				L->text[e][1][i] = rev ? comp(comp(c)) : comp(c2);   // reverse_read of strand 0
			}
		}
		wsync();
	}

	__device__ __forceinline__ void run_read(uint64_t r, uint64_t r_next)
	{
		const svg_params &p = kp->p;
		const int lane = lane_id();
		const int gap = kp->ix.gap;
		// text (fetch_next_read_pair: -S reversal), both strands, from the words prefetched
		// at the end of the previous read (or before the first)
		stage_text();
		for (int e = 0; e < ENDS; e++) {
			const int len = rc.rl[e];
			if (len >= 15 + gap) {   // shorter reads: out of contract, no hits (see oracle)
				int cr = (len - 15 - gap) << 16, step;
				if (len <= 160) {
					step = cr / (p.total_subreads - 1);
					if (step < (gap << 16)) step = gap << 16;
				} else {
					step = 6 << 16;
					if (cr / step > 62) step = cr / 62;
				}
				rc.step[e] = step;
				rc.applied[e] = 1 + cr / step;
				rc.np[e] = rc.applied[e] * gap;
				if (rc.np[e] > MAXP || rc.np[e] > kp->nps) {
					// beyond the probe records of this batch (svg_set_max_read_length) or the LDS
					// probe tables: zero records and a sticky error (svg_device_status)
					if (lane == 0) atomicOr(kp->err, 1u);
					rc.np[e] = 0; rc.applied[e] = 0;
				}
			} else {
				rc.step[e] = 0; rc.applied[e] = 0; rc.np[e] = 0;
			}
		}
		for (int e = 0; e < ENDS; e++) {
			if (kp->stored) {
				// multi-block index, block > 0: the bigtable already holds the previous blocks'
				// results, and top-K merges this block's table with them (core.c:3567-3613)
				const uint64_t q = (r * ENDS + e) * (uint64_t)p.multi_best;
				const uint32_t *src = (const uint32_t *)(kp->out + q * 68);
				if (lane < 51) L->res[e][lane / 17][lane % 17] = lane < 17 * p.multi_best ? src[lane] : 0u;
				if constexpr (SJ) {
					const uint32_t *js = kp->jout ? (const uint32_t *)(kp->jout + q * 16) : NULL;
					const uint16_t *bs = kp->bm_out ? kp->bm_out + (r * ENDS + e) * (uint64_t)SVG_BIG_MARGIN_WORDS : NULL;
					if (lane < 12) L->jres[e][lane / 4][lane % 4] = js && lane < 4 * p.multi_best ? js[lane] : 0u;
					if (lane < 10) L->bm[e][lane] = bs && lane < SVG_BIG_MARGIN_WORDS ? bs[lane] : (uint16_t)0;
				}
			} else {
				for (int i = 0; i < 3; i++) rec_zero(L->res[e][i]);
				if (lane < 12) L->jres[e][lane / 4][lane % 4] = 0;
				if (lane < 10) L->bm[e][lane] = 0;
			}
		}
		wsync();
		STAMP(0);
		stage_probes();
		// this read's text and probe records are staged: the next read's loads go out now and
		// have the whole vote of this read to arrive (deferred reads are scattered over the chunk)
		if (r_next < kp->n_reads) { prefetch_text(r_next); prefetch_recs(r_next); }
		STAMP(1);
		for (int strand = 0; strand < 2; strand++) {
			cur_strand = strand;
			vote_end<0>(strand);
			if constexpr (ENDS == 2) {
				compact_end0();
				vote_end<1>(strand);
			}
			STAMP(3);
			// (one call site: a second one kept topk out of line, and the wave's state in scratch)
			if (ENDS == 2 || max_vote[0] >= p.min_votes_first) topk(strand);
			else if (rec_votes(L->res[0][0]) < 1) {
				if (lane == 0) {
					uint32_t *r0 = L->res[0][0];
					rec_set_noninf(r0, 0);
					if (rc.applied[0] > rec_used(r0)) rec_set_used(r0, rc.applied[0]);
				}
				wsync();
			}
			STAMP(4);
		}
		// write the read's records (multi_best <= 3: 17 * 3 dwords, one store per lane)
		for (int e = 0; e < ENDS; e++) {
			uint32_t *dst = (uint32_t *)(kp->out + ((r * ENDS + e) * (uint64_t)p.multi_best) * 68);
			if (lane < 17 * p.multi_best) dst[lane] = L->res[e][lane / 17][lane % 17];
		}
		if constexpr (SJ) {
			for (int e = 0; e < ENDS; e++) {
				if (p.do_breakpoint_detection) {
					uint32_t *jd = (uint32_t *)(kp->jout + ((r * ENDS + e) * (uint64_t)p.multi_best) * 16);
					if (lane < 4 * p.multi_best) jd[lane] = L->jres[e][lane / 4][lane % 4];
				}
				if (p.do_big_margin_filtering_for_junctions) {
					uint16_t *bd = kp->bm_out + (r * ENDS + e) * (uint64_t)SVG_BIG_MARGIN_WORDS;
					if (lane < SVG_BIG_MARGIN_WORDS) bd[lane] = L->bm[e][lane];
				}
			}
		}
		if (kp->stats) {
			for (int e = 0; e < ENDS; e++)
				for (int i = 0; i < p.multi_best; i++)
					if (lane == 0 && rec_votes(L->res[e][i]) > 0) atomicAdd(&kp->stats[3], 1ull);
		}
		wsync();
	}
};

template <int ENDS, int MAXL, int MAXP, int WPB, int OCC, bool SJ>
__global__ void __launch_bounds__(64 * WPB, OCC) vote_kernel(KParams kp)
{
	extern __shared__ __align__(16) uint8_t lds_raw[];
	typedef WaveLDS<ENDS, MAXL, MAXP, SJ> LT;
	// wave-uniform values are made scalar (readfirstlane) so that the wave's pointers and its read
	// loop state live in SGPRs: in VGPRs they were the first things spilled around run_read (12
	// scratch stores per read in the 80-VGPR single-end build)
	const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
	const uint64_t gw = (uint64_t)blockIdx.x * WPB + wib;
	const uint64_t nw = (uint64_t)gridDim.x * WPB;
	Wave<ENDS, MAXL, MAXP, SJ> W;
	W.L = reinterpret_cast<LT *>(lds_raw + (size_t)wib * ((sizeof(LT) + 15) & ~(size_t)15));
	W.kp = &kp;
	const size_t per_end = (size_t)NSLOT * COLD_WORDS + NSLOT;   // cold + shift_locs
	const size_t per_wave = per_end * ENDS + (ENDS == 2 ? (size_t)NSLOT * 4 : 0);   // + PE overflow list
	uint32_t *base = kp.scratch + gw * per_wave;
	for (int e = 0; e < ENDS; e++) {
		W.cold[e] = base + e * per_end;
		W.shift_locs[e] = base + e * per_end + (size_t)NSLOT * COLD_WORDS;
	}
	W.ovf = base + per_end * ENDS;
#ifdef SVG_STAMPS
	for (int k = 0; k < 12; k++) W.acc[k] = 0;
	for (int k = 0; k < 4; k++) W.why[k] = 0;
	W.t_last = __builtin_amdgcn_s_memtime();
#endif
	// direct: reads gw, gw+nw, ...; indirect: the deferred reads idx[pos].  Deferred reads differ
	// widely in cost (repeat families): the first static_eighths / 8 of the list are dealt out
	// statically (positions gw, gw+nw, ... below n_static: no atomic), the rest come from the work
	// counter, one read ahead (the atomic's result is consumed a whole read later).  Each loop
	// trip knows the current and the next position; the next read's index is needed for its
	// prefetch (run_read), the position after it is computed or requested during the read.
	const uint64_t n = kp.idx ? (uint64_t)*kp.idx_count : kp.n_reads;
	const uint64_t n_static = kp.idx ? (n * (uint64_t)kp.static_eighths / 8) / nw * nw : n;
	auto grab = [&]() -> uint64_t {   // a dynamic position, synchronously (twice per wave at most)
		uint32_t a = 0;
		if (lane_id() == 0) a = atomicAdd(kp.work, 1u);
		return n_static + (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)a, 0));
	};
	auto uni = [](uint64_t v) -> uint64_t {   // a wave-uniform 64-bit value, scalar
		return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
		       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
	};
	auto dyn_after = [&](uint64_t p) { return kp.idx && p + nw >= n_static; };   // p's successor is dynamic
	uint64_t i = !kp.idx || gw < n_static ? gw : (n ? grab() : n);
	uint64_t in = i >= n ? n : (dyn_after(i) ? grab() : i + nw);
	uint64_t r = uni(i < n ? (kp.idx ? kp.idx[i] : i) : 0);
	if (i < n) { W.prefetch_text(r); W.prefetch_recs(r); }
	while (i < n) {
		const bool dyn = in < n && dyn_after(in);
		uint32_t nxt = 0;
		if (dyn && lane_id() == 0) nxt = atomicAdd(kp.work, 1u);   // consumed after this read
		const uint64_t rn = uni(in < n ? (kp.idx ? kp.idx[in] : in) : kp.n_reads);
		W.run_read(r, rn);
		const uint64_t in2 = in >= n ? n : (dyn ? n_static + (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)nxt, 0)) : in + nw);
		i = in;
		r = rn;
		in = in2;
#ifdef SVG_STAMPS
		{ unsigned long long _t = __builtin_amdgcn_s_memtime(); W.acc[5] += _t - W.t_last; W.t_last = _t; }
#endif
	}
#ifdef SVG_STAMPS
	if (kp.stats && lane_id() == 0) {
		for (int k = 0; k < 8; k++) atomicAdd(&kp.stats[8 + k], W.acc[k]);
		for (int k = 8; k < 12; k++) atomicAdd(&kp.stats[21 + k - 8], W.acc[k]);
		for (int k = 0; k < 4; k++) atomicAdd(&kp.stats[28 + k], W.why[k]);
	}
#endif
	// (stats: results [3], batch-settled / serially replayed candidates [26] / [27] are added where
	// they happen; probes, bucket items and hits [0..2] by the probe kernels)
}

// equal-key run of a bucket given as a bit mask over its items: gehash_go_X's binary search
// (sorted-hashtable.c:947-981) replayed on the positions alone -- it stops at the first
// midpoint inside the run.  False (caller falls back to the key loop) if the run is not
// contiguous, i.e. the bucket is not sorted.
__device__ __forceinline__ bool try_run(uint64_t eq, int n, int &m, int &fwd, int &bwd, bool &hit)
{
	const int fe = eq ? __builtin_ctzll(eq) : 0, ne = __popcll(eq);
	if (eq && eq != (((ne == 64 ? 0ull : (1ull << ne)) - 1ull) << fe)) return false;
	if (eq) {
		const int le = fe + ne - 1;
		int lo = 0, hi = n - 1;
		for (;;) {
			m = (lo + hi) >> 1;
			if (m < fe) lo = m + 1;
			else if (m > le) hi = m - 1;
			else break;
		}
		hit = true;
		fwd = le - m + 1;
		bwd = m - fe;
	}
	return true;
}

// 16-mer key of probe p (subread x gap slot) of strand s of end e of read r (genekey2int,
// input-files.c:1232, at the subread offset of core.c:3117-3171); false if the read has no
// such probe (shorter than 15 + gap, or p beyond its applied subreads)
template <int ENDS, bool PACKED>
__device__ __forceinline__ bool probe_key(const PParams &pp, uint32_t r, int e, int s, int p, uint32_t &key)
{
	int len = e ? pp.len2[r] : pp.len1[r];
	if (len > SVG_READ_KEEP) len = SVG_READ_KEEP;
	const int gap = pp.ix.gap;
	if (len < 15 + gap) return false;
	const int cr = (len - 15 - gap) << 16;
	int step;
	if (len <= 160) { step = cr / (pp.total_subreads - 1); if (step < (gap << 16)) step = gap << 16; }
	else { step = 6 << 16; if (cr / step > 62) step = cr / 62; }
	const int np = (1 + cr / step) * gap;
	if (p >= np) return false;
	const int k = p / gap, x = p - k * gap;
	int off = (int)(((int64_t)step * k) >> 16);
	if (gap > 1) off -= off % gap - x;
	// 16 bases of strand s at off; strand 1 = reverse_read of strand 0, strand 0 = the input,
	// reverse-complemented for -S (R2 by default)
	const int rev = e ? pp.reverse_r2 : pp.reverse_r1;
	const bool direct = s == rev;
	const int start = direct ? off : len - 16 - off;
	key = 0;
	if constexpr (PACKED) {
		// 2-bit input (svg_packed_reads): the 16 codes at base k0 are one 32-bit window,
		// already genekey2int's key.  Reverse strand: complement (~code; an exception base
		// complements to 'N' = 3) and reverse the 2-bit groups.  Strand 1 of a reversed
		// read is comp(comp(input)): the codes, with exception bases turned into 'N'.
		const uint64_t k0 = (pp.pk_starts[e] ? pp.pk_starts[e][r] : pp.pk_base0[e] + (uint64_t)r * pp.pk_stride[e]) +
		                    (uint64_t)start;
		const uint32_t *bw = pp.pk_bases[e] + (k0 >> 4);
		const uint32_t s2 = 2u * (uint32_t)(k0 & 15u);
		const uint32_t W = s2 ? (bw[0] << s2) | (bw[1] >> (32u - s2)) : bw[0];
		uint32_t X2 = 0;
		if (pp.pk_xmask[e]) {
			const uint32_t *xw = pp.pk_xmask[e] + (k0 >> 5);
			const uint32_t s1 = (uint32_t)(k0 & 31u);
			// bases k0..k0+15 (the next word only when they reach into it)
			uint32_t t = (s1 > 16u ? (xw[0] << s1) | (xw[1] >> (32u - s1)) : xw[0] << s1) >> 16;
			t = (t | (t << 8)) & 0x00ff00ffu;
			t = (t | (t << 4)) & 0x0f0f0f0fu;
			t = (t | (t << 2)) & 0x33333333u;
			t = (t | (t << 1)) & 0x55555555u;
			X2 = t | (t << 1);   // base i -> bits 31-2i .. 30-2i
		}
		if (direct) key = (s == 1 && rev) ? (W | X2) : W;
		else {
			const uint32_t v = __builtin_bitreverse32(~W | X2);
			key = ((v >> 1) & 0x55555555u) | ((v & 0x55555555u) << 1);
		}
	} else {
		const char *src = (e ? pp.seq2 : pp.seq1) + (e ? pp.off2[r] : pp.off1[r]) + start;
		const uintptr_t a = (uintptr_t)src;
		const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
		const int sh = (int)(a & 3);
		uint32_t wd[5];
#pragma unroll
		for (int q = 0; q < 4; q++) wd[q] = w[q];
		wd[4] = sh ? w[4] : 0u;   // only when the window reaches into it
#pragma unroll
		for (int i = 0; i < 16; i++) {
			const int bi = sh + (direct ? i : 15 - i);
			char c = (char)((wd[bi >> 2] >> (8 * (bi & 3))) & 0xff);
			if (!direct) c = comp(c);
			if (s == 1 && rev) c = comp(comp(c));   // strand 1 of a reversed read: comp(comp(input))
			key |= b2i(c) << (30 - 2 * i);
		}
	}
	return true;
}

// =============================================================================================
// probe kernel: phase P for a whole chunk of reads, one thread per subread probe.  Same
// arithmetic as Wave::probe_all (genekey2int, key % nb, gehash_go_X's binary search and the
// equal-key run on both sides of the first-hit midpoint); with no per-read state to keep,
// it runs at high occupancy and hides the dependent bucket -> keys -> run chain.
// =============================================================================================
template <int ENDS, int BPC, bool LINE, bool PACKED>
__global__ void __launch_bounds__(256, BPC) probe_kernel(PParams pp)
{
	const DevIndex &ix = pp.ix;
	const uint32_t nps = (uint32_t)pp.nps, per_read = ENDS * 2 * nps;
	const uint32_t total = pp.n_reads * per_read;
	const int gap = ix.gap;
	unsigned long long st_p = 0, st_i = 0, st_h = 0;
	// each block walks one contiguous range of 256-probe tiles: blocks are dealt round-robin to
	// the 8 XCDs, so a grid-stride walk would put neighbouring reads (which share the lines of
	// the SoA record rows) on different L2s and turn every record store into a partial-line write
	const uint32_t tiles = (total + 255u) / 256u, per_blk = (tiles + gridDim.x - 1u) / gridDim.x;
	const uint32_t tile_end = min(tiles, (blockIdx.x + 1u) * per_blk);
	for (uint32_t tile = blockIdx.x * per_blk; tile < tile_end; tile++) {
		const uint32_t t = tile * 256u + threadIdx.x;
		if (t >= total) break;
		uint32_t r, rem;
		if (pp.soa && !pp.readmajor) { rem = t / pp.n_reads; r = t - rem * pp.n_reads; }
		else { r = t / per_read; rem = t - r * per_read; }
		const int e = ENDS == 2 ? (int)(rem / (2 * nps)) : 0;
		const uint32_t rem2 = rem - (uint32_t)e * 2 * nps;
		const int s = rem2 >= nps ? 1 : 0;
		const int p = (int)(rem2 - (uint32_t)s * nps);
		uint2 rec = make_uint2(0u, 0u);
		uint32_t key;
		if (probe_key<ENDS, PACKED>(pp, r, e, s, p, key)) {
			{
				const uint32_t q = (uint32_t)__umul64hi((uint64_t)key, pp.nb_magic);
				const uint32_t b = key - q * ix.nb;
				const int16_t k16 = (int16_t)q;
				uint32_t first;
				int n;
				bool compact = false, inl = false;
				uint4 lw[4];
				if constexpr (LINE) {
					// the bucket's 64-byte line: bounds and u8 keys in one random access
					const uint4 *l4 = ix.bline + 4 * (size_t)b;
#pragma unroll
					for (int q = 0; q < 4; q++) lw[q] = l4[q];
					const uint32_t c = lw[0].y & 255u;
					first = lw[0].x;
					n = (int)c;
					compact = c != 255u;
					inl = c <= 59u;
				} else if (ix.bgrp) {
					// bucket bounds from the 32-byte group: first item of the group + the counts
					// of the buckets before b in it
					const uint4 *g4 = (const uint4 *)(ix.bgrp + 8 * (size_t)(b >> 4));
					const uint4 ga = g4[0], gb = g4[1];
					const uint32_t i = b & 15u;
					const uint32_t cw[4] = {ga.y, ga.z, ga.w, gb.x};
					uint32_t pre = 0;
					bool sat = false;   // a bucket before b in the group has 255+ items: its byte is no count
#pragma unroll
					for (int q = 0; q < 4; q++) {
						// bytes of word q below i
						const int nb_ = (int)i - 4 * q;
						const uint32_t msk = nb_ >= 4 ? 0xffffffffu : nb_ <= 0 ? 0u : (1u << (8 * nb_)) - 1u;
						pre = __builtin_amdgcn_sad_u8(cw[q] & msk, 0u, pre);
						const uint32_t t = ~cw[q] | ~msk;   // zero byte <=> a 0xff count below i
						sat |= ((t - 0x01010101u) & ~t & 0x80808080u) != 0u;
					}
					const uint32_t wsel = i < 4 ? ga.y : i < 8 ? ga.z : i < 12 ? ga.w : gb.x;
					const uint32_t c = (wsel >> (8 * (i & 3u))) & 255u;
					first = ga.x + pre;
					n = (int)c;
					compact = c != 255u && !sat;
				}
				if (!compact) {
					first = ix.bstart[b];
					n = (int)(ix.bstart[b + 1] - first);
				}
				st_p++;
				st_i += (unsigned)n;
				if (n > 0) {
					const int16_t *K = ix.keys + first;
					int m = 0, fwd = 0, bwd = 0;
					bool hit = false, done = false;
					if (LINE && inl) {
						// u8 keys at bytes 5..63 of the line, equal keys by a zero-byte test
						const uint32_t kk = (uint32_t)(uint8_t)k16 * 0x01010101u;
						uint64_t eq = 0;
#pragma unroll
						for (int k = 0; k < 4; k++) {
							const uint32_t dw[4] = {lw[k].x, lw[k].y, lw[k].z, lw[k].w};
#pragma unroll
							for (int q = 0; q < 4; q++) {
								const uint32_t x = dw[q] ^ kk;
								const uint32_t z = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
								const uint32_t bits = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
								eq |= (uint64_t)bits << (16 * k + 4 * q);
							}
						}
						eq = (eq >> 5) & ((1ull << n) - 1ull);
						done = try_run(eq, n, m, fwd, bwd, hit);
					} else if (!LINE && compact && n <= 48) {
						// u8 keys: the bucket in <= 4 independent 16-byte loads, equal keys by a
						// zero-byte test
						const uintptr_t base = (uintptr_t)(ix.keys8 + first);
						const uint4 *w = (const uint4 *)(base & ~(uintptr_t)15);
						const int sh = (int)(base & 15);
						const int nq = (sh + n + 15) >> 4;
						const uint32_t kk = (uint32_t)(uint8_t)k16 * 0x01010101u;
						uint64_t eq = 0;
#pragma unroll
						for (int k = 0; k < 4; k++) {
							const uint4 v = k < nq ? w[k] : make_uint4(0u, 0u, 0u, 0u);
							const uint32_t dw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
							for (int q = 0; q < 4; q++) {
								const uint32_t x = dw[q] ^ kk;
								const uint32_t z = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
								const uint32_t bits = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
								eq |= (uint64_t)bits << (16 * k + 4 * q);
							}
						}
						eq = (eq >> sh) & ((1ull << n) - 1ull);
						done = try_run(eq, n, m, fwd, bwd, hit);
					} else if (!LINE && pp.window && n <= 56) {
						// i16 keys: <= 8 independent 16-byte loads of the aligned window holding the
						// bucket, equal keys by a zero-halfword test
						const uintptr_t base = (uintptr_t)K;
						const uint4 *w = (const uint4 *)(base & ~(uintptr_t)15);
						const int sh = (int)((base & 15) >> 1);   // halfword of item 0 in the window
						const int nq = (sh + n + 7) >> 3;         // 16-byte words holding the bucket
						const uint32_t kk = (uint32_t)(uint16_t)k16 * 0x00010001u;
						uint64_t eq = 0;
#pragma unroll
						for (int k = 0; k < 8; k++) {
							const uint4 v = k < nq ? w[k] : make_uint4(0u, 0u, 0u, 0u);
							const uint32_t dw[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
							for (int q = 0; q < 4; q++) {
								const uint32_t x = dw[q] ^ kk;
								const uint32_t z = ~(((x & 0x7fff7fffu) + 0x7fff7fffu) | x | 0x7fff7fffu);
								const int j = 4 * k + q;
								eq |= ((uint64_t)((z >> 15) & 1u) << (2 * j)) | ((uint64_t)(z >> 31) << (2 * j + 1));
							}
						}
						eq = (eq >> sh) & ((1ull << n) - 1ull);
						done = try_run(eq, n, m, fwd, bwd, hit);
					}
					if (!done) {
						int lo = 0, hi = n - 1;
						for (;;) {
							m = (lo + hi) >> 1;
							int16_t kk = K[m];
							if (kk > k16) hi = m - 1;
							else if (kk < k16) lo = m + 1;
							else { hit = true; break; }
							if (hi < lo) break;
						}
						if (hit) {
							int qq = m + 1;
							while (qq < n && K[qq] == k16) qq++;
							fwd = qq - m;
							qq = m - 1;
							while (qq >= 0 && K[qq] == k16) qq--;
							bwd = m - 1 - qq;
						}
					}
					if (hit) {
						rec = make_uint2(first + (uint32_t)m, (uint32_t)fwd | ((uint32_t)bwd << 16));
						st_h += (unsigned)(fwd + bwd);
					}
				}
			}
		}
		pp.out[pp.soa ? (size_t)rem * pp.n_reads + r : (size_t)t] = rec;
	}
	if (pp.stats) {
		for (int o = 32; o; o >>= 1) {
			st_p += __shfl_xor(st_p, o); st_i += __shfl_xor(st_i, o); st_h += __shfl_xor(st_h, o);
		}
		if (lane_id() == 0 && st_p) {
			atomicAdd(&pp.stats[0], st_p);
			atomicAdd(&pp.stats[1], st_i);
			atomicAdd(&pp.stats[2], st_h);
		}
	}
}

// =============================================================================================
// bucket-line probe kernel (indexes with the 64-B bucket-line image: every -F -B index):
//   * reads in groups of pp.group (group * per_read <= PROBE_GROUP_RECS probes): a group's
//     records are staged in LDS and leave as whole rows ([row][read], SoA) or one contiguous
//     range (AoS) instead of one scattered 8-byte store per probe;
//   * a probe whose bucket holds more than 59 items -- no room for its keys in the line; at C3
//     the repeat-family buckets -- does not search here: it leaves its key in its record slot
//     (marked fwd = bwd = 0xffff) and its slot index in a list, and probe_big_kernel searches
//     those 32 lanes per probe.  Before this split one such probe held its whole wave in a
//     dependent binary search plus a one-load-per-step run scan.
// =============================================================================================
#define PROBE_GROUP_RECS 2048
#define IMG_LINE  0
#define IMG_CODE  1
#define IMG_KHASH 2
// probes per thread and pass of the code / key-hash line kernels (their loads in flight
// together): 2 -- C3 0.976 -> 0.913 ms per launch, 469.6 Mreads/s (profiles/r04/bench_c3_probe2.json);
// 3 measured the same (0.920 ms, 467.0, bench_c3_r4i.json) and 4 spills 46 registers at 8 waves/SIMD
template <int ENDS, bool PACKED>
struct ProbeDepth { static constexpr int value = 2; };

// a probe's record from its bucket's 32-byte code (q: key / nb, the key_hi the code counts):
// the equal-key run's bounds by two selects on the code's zero bits, gehash_go_X's binary search
// replayed on them for the first-hit midpoint; count byte 255 = the big-bucket list
__device__ __forceinline__ void code_record(const uint4 u0, const uint4 u1, uint32_t q, uint32_t key, uint2 &rec, bool &big,
                                            unsigned long long &st_i, unsigned long long &st_h)
{
	const uint32_t c = u0.y & 255u, first = u0.x;
	big = c == 255u;
	if (!big && c) {
		const uint64_t z[4] = {~(((uint64_t)u0.y << 32) | u0.x) & ~0xffffffffffull, ~(((uint64_t)u0.w << 32) | u0.z),
		                       ~(((uint64_t)u1.y << 32) | u1.x), ~(((uint64_t)u1.w << 32) | u1.z)};
		const int k = (int)q;
		const int fe = k ? code_zero(z, k - 1) - 40 - (k - 1) : 0;
		const int ee = code_zero(z, k) - 40 - k;   // items with key_hi <= k
		st_i += c;
		if (ee > fe) {
			const int le = ee - 1;
			int lo = 0, hi = (int)c - 1, m;
			for (;;) {
				m = (lo + hi) >> 1;
				if (m < fe) lo = m + 1;
				else if (m > le) hi = m - 1;
				else break;
			}
			rec = make_uint2(first + (uint32_t)m, (uint32_t)(le - m + 1) | ((uint32_t)(m - fe) << 16));
			st_h += (unsigned)(ee - fe);
		}
	}
	if (big) rec = make_uint2(key, 0xffffffffu);
}

template <int ENDS, bool PACKED, int IMG>
__global__ void __launch_bounds__(256, 8) probe_line_kernel(PParams pp)
{
	__shared__ uint2 srec[PROBE_GROUP_RECS];
	__shared__ uint32_t s_big;   // entries of this block's region of the big-bucket list
	const DevIndex &ix = pp.ix;
	const uint32_t nps = (uint32_t)pp.nps, per_read = ENDS * 2 * nps, n = pp.n_reads, G = pp.group;
	const uint32_t ngroups = (n + G - 1) / G, per_blk = (ngroups + gridDim.x - 1) / gridDim.x;
	const uint32_t g_end = min(ngroups, (blockIdx.x + 1) * per_blk);
	uint32_t *const big_list = pp.big_list + (size_t)blockIdx.x * pp.big_stride;
	unsigned long long st_p = 0, st_i = 0, st_h = 0;
	if (threadIdx.x == 0) s_big = 0;
	__syncthreads();
	// contiguous group ranges per block: neighbouring reads stay on one XCD's L2
	for (uint32_t g = blockIdx.x * per_blk; g < g_end; g++) {
		const uint32_t r0 = g * G, nr = min(G, n - r0), np = nr * per_read, npr = (np + 255u) & ~255u;
		// bucket code: ProbeDepth<ENDS, PACKED>::value probes per thread and pass -- their keys, then their 32-byte code loads
		// in flight together, then their decodes (the decode's selects and search replay no longer
		// sit between one probe's load and the next one's)
		if constexpr (IMG == IMG_CODE) for (uint32_t i0 = threadIdx.x; i0 < npr; i0 += 256u * ProbeDepth<ENDS, PACKED>::value) {
			uint32_t key[ProbeDepth<ENDS, PACKED>::value], outidx[ProbeDepth<ENDS, PACKED>::value], q[ProbeDepth<ENDS, PACKED>::value];
			bool ok[ProbeDepth<ENDS, PACKED>::value];
#pragma unroll
			for (int t = 0; t < ProbeDepth<ENDS, PACKED>::value; t++) {
				const uint32_t i = i0 + 256u * (uint32_t)t;
				key[t] = outidx[t] = q[t] = 0u;
				ok[t] = false;
				if (i < np) {
					const uint32_t rl = i / per_read, rem = i - rl * per_read, r = r0 + rl;
					const int e = ENDS == 2 ? (int)(rem / (2 * nps)) : 0;
					const uint32_t rem2 = rem - (uint32_t)e * 2 * nps;
					const int s = rem2 >= nps ? 1 : 0;
					const int p = (int)(rem2 - (uint32_t)s * nps);
					outidx[t] = pp.soa ? rem * n + r : r * per_read + rem;
					ok[t] = probe_key<ENDS, PACKED>(pp, r, e, s, p, key[t]);
				}
			}
			uint4 u0[ProbeDepth<ENDS, PACKED>::value], u1[ProbeDepth<ENDS, PACKED>::value];
#pragma unroll
			for (int t = 0; t < ProbeDepth<ENDS, PACKED>::value; t++) {
				u0[t] = u1[t] = make_uint4(0u, 0u, 0u, 0u);
				if (ok[t]) {
					q[t] = (uint32_t)__umul64hi((uint64_t)key[t], pp.nb_magic);
					const uint4 *c4 = ix.bcode + 2 * (size_t)(key[t] - q[t] * ix.nb);
					u0[t] = c4[0];
					u1[t] = c4[1];
				}
			}
#pragma unroll
			for (int t = 0; t < ProbeDepth<ENDS, PACKED>::value; t++) {
				const uint32_t i = i0 + 256u * (uint32_t)t;
				if (i - threadIdx.x >= npr) break;   // block-uniform (npr is a multiple of 256)
				uint2 rec = make_uint2(0u, 0u);
				bool big = false;
				if (ok[t]) {
					st_p++;
					code_record(u0[t], u1[t], q[t], key[t], rec, big, st_i, st_h);
				}
				const unsigned long long bm = ballot(big);
				if (bm) {
					const int leader = __ffsll((long long)bm) - 1;
					uint32_t base = 0;
					if (lane_id() == leader) base = atomicAdd(&s_big, (uint32_t)__popcll(bm));
					base = __shfl(base, leader);
					if (big) big_list[base + lanes_below(bm)] = outidx[t];
				}
				if (i < np) srec[i] = rec;
			}
		}
		// key-hash image in 32-byte sectors: the same pass (the probes' first sectors in flight
		// together; an overflow chain continues from the next sector)
		if (IMG == IMG_KHASH && ix.khash_sec) for (uint32_t i0 = threadIdx.x; i0 < npr; i0 += 256u * ProbeDepth<ENDS, PACKED>::value) {
			uint32_t key[ProbeDepth<ENDS, PACKED>::value], outidx[ProbeDepth<ENDS, PACKED>::value];
			uint64_t L[ProbeDepth<ENDS, PACKED>::value];
			bool ok[ProbeDepth<ENDS, PACKED>::value];
#pragma unroll
			for (int t = 0; t < ProbeDepth<ENDS, PACKED>::value; t++) {
				const uint32_t i = i0 + 256u * (uint32_t)t;
				key[t] = outidx[t] = 0u;
				L[t] = 0u;
				ok[t] = false;
				if (i < np) {
					const uint32_t rl = i / per_read, rem = i - rl * per_read, r = r0 + rl;
					const int e = ENDS == 2 ? (int)(rem / (2 * nps)) : 0;
					const uint32_t rem2 = rem - (uint32_t)e * 2 * nps;
					const int s = rem2 >= nps ? 1 : 0;
					const int p = (int)(rem2 - (uint32_t)s * nps);
					outidx[t] = pp.soa ? rem * n + r : r * per_read + rem;
					ok[t] = probe_key<ENDS, PACKED>(pp, r, e, s, p, key[t]);
				}
			}
			uint4 a[ProbeDepth<ENDS, PACKED>::value], b4[ProbeDepth<ENDS, PACKED>::value];
#pragma unroll
			for (int t = 0; t < ProbeDepth<ENDS, PACKED>::value; t++) {
				a[t] = b4[t] = make_uint4(0u, 0u, 0u, 0u);
				if (ok[t] && key[t] != 0xffffffffu) {
					L[t] = khash_line(key[t], ix.khash_lines);
					const uint4 *l4 = (const uint4 *)(ix.khash + 8 * L[t]);
					a[t] = l4[0];
					b4[t] = l4[1];
				}
			}
#pragma unroll
			for (int t = 0; t < ProbeDepth<ENDS, PACKED>::value; t++) {
				const uint32_t i = i0 + 256u * (uint32_t)t;
				if (i - threadIdx.x >= npr) break;   // block-uniform
				uint2 rec = make_uint2(0u, 0u);
				if (ok[t]) {
					st_p++;
					if (pp.stats) {
						const uint32_t q = (uint32_t)__umul64hi((uint64_t)key[t], pp.nb_magic), b = key[t] - q * ix.nb;
						st_i += ix.bstart[b + 1] - ix.bstart[b];
					}
					if (key[t] == 0xffffffffu) khash_find(ix, key[t], rec);
					else {
						bool more;
						if (!khash_sector(a[t], b4[t], key[t], rec, more) && more)
							khash_find_from(ix, key[t], L[t] + 1 == ix.khash_lines ? 0 : L[t] + 1, rec);
					}
					if (pp.stats) st_h += (rec.y & 0xffffu) + (rec.y >> 16);
				}
				if (i < np) srec[i] = rec;   // (the key-hash image has no big-bucket list)
			}
		}
		if (IMG != IMG_CODE && !(IMG == IMG_KHASH && ix.khash_sec)) for (uint32_t i = threadIdx.x; i < npr; i += 256u) {
			uint2 rec = make_uint2(0u, 0u);
			bool big = false;
			uint32_t outidx = 0;
			if (i < np) {
				const uint32_t rl = i / per_read, rem = i - rl * per_read, r = r0 + rl;
				const int e = ENDS == 2 ? (int)(rem / (2 * nps)) : 0;
				const uint32_t rem2 = rem - (uint32_t)e * 2 * nps;
				const int s = rem2 >= nps ? 1 : 0;
				const int p = (int)(rem2 - (uint32_t)s * nps);
				outidx = pp.soa ? rem * n + r : r * per_read + rem;
				uint32_t key;
				if (IMG == IMG_KHASH && probe_key<ENDS, PACKED>(pp, r, e, s, p, key)) {
					// the key's record from its 64-byte line (and the overflow chain)
					st_p++;
					if (pp.stats) {
						const uint32_t q = (uint32_t)__umul64hi((uint64_t)key, pp.nb_magic), b = key - q * ix.nb;
						st_i += ix.bstart[b + 1] - ix.bstart[b];
					}
					khash_find(ix, key, rec);
					if (pp.stats) st_h += (rec.y & 0xffffu) + (rec.y >> 16);
				} else if (IMG == IMG_LINE && probe_key<ENDS, PACKED>(pp, r, e, s, p, key)) {
					const uint32_t q = (uint32_t)__umul64hi((uint64_t)key, pp.nb_magic);
					const uint32_t b = key - q * ix.nb;
					// the bucket's 64-byte line: bounds and u8 keys in one random access
					const uint4 *l4 = ix.bline + 4 * (size_t)b;
					uint4 lw[4];
#pragma unroll
					for (int k = 0; k < 4; k++) lw[k] = l4[k];
					const uint32_t c = lw[0].y & 255u, first = lw[0].x;
					st_p++;
					big = c > 59u;
					if (!big && c) {
						// u8 keys at bytes 5..63 of the line, equal keys by a zero-byte test
						const uint32_t kk = (uint32_t)(uint8_t)q * 0x01010101u;
						uint64_t eq = 0;
#pragma unroll
						for (int k = 0; k < 4; k++) {
							const uint32_t dw[4] = {lw[k].x, lw[k].y, lw[k].z, lw[k].w};
#pragma unroll
							for (int qq = 0; qq < 4; qq++) {
								const uint32_t x = dw[qq] ^ kk;
								const uint32_t z = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
								const uint32_t bits = ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
								eq |= (uint64_t)bits << (16 * k + 4 * qq);
							}
						}
						eq = (eq >> 5) & ((1ull << c) - 1ull);
						int m = 0, fwd = 0, bwd = 0;
						bool hit = false;
						if (try_run(eq, (int)c, m, fwd, bwd, hit)) {
							st_i += c;
							if (hit) {
								rec = make_uint2(first + (uint32_t)m, (uint32_t)fwd | ((uint32_t)bwd << 16));
								st_h += (unsigned)(fwd + bwd);
							}
						} else big = true;   // unsorted bucket: the literal search, in probe_big_kernel
					}
					if (big) rec = make_uint2(key, 0xffffffffu);
				}
			}
			// the block's region of the big-bucket list: one LDS atomic per wave (a single global
			// counter for the whole grid serialised ~2M atomics per launch)
			const unsigned long long bm = ballot(big);
			if (bm) {
				const int leader = __ffsll((long long)bm) - 1;
				uint32_t base = 0;
				if (lane_id() == leader) base = atomicAdd(&s_big, (uint32_t)__popcll(bm));
				base = __shfl(base, leader);
				if (big) big_list[base + lanes_below(bm)] = outidx;
			}
			if (i < np) srec[i] = rec;
		}
		__syncthreads();
		for (uint32_t i = threadIdx.x; i < np; i += 256u) {
			if (pp.soa) {
				const uint32_t row = i / nr, rl = i - row * nr;
				pp.out[(size_t)row * n + r0 + rl] = srec[rl * per_read + row];
			} else pp.out[(size_t)r0 * per_read + i] = srec[i];
		}
		__syncthreads();
	}
	if (threadIdx.x == 0) pp.big_count[blockIdx.x] = s_big;
	if (pp.stats) {
		for (int o = 32; o; o >>= 1) {
			st_p += __shfl_xor(st_p, o); st_i += __shfl_xor(st_i, o); st_h += __shfl_xor(st_h, o);
		}
		if (lane_id() == 0 && st_p) {
			atomicAdd(&pp.stats[0], st_p);
			atomicAdd(&pp.stats[1], st_i);
			atomicAdd(&pp.stats[2], st_h);
		}
	}
}

// The big-bucket probes of probe_line_kernel, 8 lanes per probe: in each pass lane j loads the
// 16-byte word 8*pass+j of the aligned window holding the bucket's i16 keys (8 keys, one 128-B
// row per 8 lanes; up to four passes = 256 items in flight at once), the 8 lanes reduce first /
// last / count of the equal keys, and gehash_go_X's binary search (sorted-hashtable.c:947-981)
// is replayed on the run's positions to get the reference's first-hit midpoint.  A bucket
// whose equal keys are not one run (not sorted) takes the literal search.
__global__ void __launch_bounds__(256) probe_big_kernel(PParams pp)
{
	const DevIndex &ix = pp.ix;
	const int sub = (int)(threadIdx.x & 7u);
	unsigned long long st_i = 0, st_h = 0, st_n = 0;
	// list regions of the line kernel's blocks (pp.big_regions of them)
	for (uint32_t reg = blockIdx.x; reg < pp.big_regions; reg += gridDim.x) {
		const uint32_t cnt = pp.big_count[reg];
		const uint32_t *list = pp.big_list + (size_t)reg * pp.big_stride;
		st_n += threadIdx.x == 0 ? cnt : 0u;
		for (uint32_t j = threadIdx.x >> 3; j < cnt; j += 32u) {
			const uint32_t outidx = list[j];
			const uint32_t key = pp.out[outidx].x;
			const uint32_t q = (uint32_t)__umul64hi((uint64_t)key, pp.nb_magic);
			const uint32_t b = key - q * ix.nb;
			const uint16_t k16 = (uint16_t)q;
			const uint2 l0 = ix.bcode ? *(const uint2 *)(ix.bcode + 2 * (size_t)b) : *(const uint2 *)(ix.bline + 4 * (size_t)b);
			const uint32_t first = l0.x;
			uint32_t nn = l0.y & 255u;
			if (nn == 255u) nn = ix.bstart[b + 1] - first;   // 255 = not in the image (or 255+ items)
			const int16_t *K = ix.keys + first;
			const uint4 *W = (const uint4 *)((uintptr_t)K & ~(uintptr_t)15);
			const int sh = (int)(((uintptr_t)K & 15) >> 1);   // item 0 is halfword sh of word 0
			const int nw = (sh + (int)nn + 7) >> 3;           // 16-byte words holding the bucket
			int fe = 0x7fffffff, le = -1, ne = 0;
			for (int w0 = 0; w0 < nw; w0 += 32) {
				uint4 v[4];
#pragma unroll
				for (int ps = 0; ps < 4; ps++) {
					const int w = w0 + 8 * ps + sub;
					v[ps] = w < nw ? W[w] : make_uint4(0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu);
				}
#pragma unroll
				for (int ps = 0; ps < 4; ps++) {
					const int w = w0 + 8 * ps + sub;
					const uint32_t dw[4] = {v[ps].x, v[ps].y, v[ps].z, v[ps].w};
#pragma unroll
					for (int h = 0; h < 8; h++) {
						const int it = 8 * w + h - sh;
						if (it >= 0 && it < (int)nn && (uint16_t)(dw[h >> 1] >> (16 * (h & 1))) == k16) {
							fe = min(fe, it); le = max(le, it); ne++;
						}
					}
				}
			}
#pragma unroll
			for (int o = 4; o; o >>= 1) {
				fe = min(fe, __shfl_xor(fe, o));
				le = max(le, __shfl_xor(le, o));
				ne += __shfl_xor(ne, o);
			}
			uint2 rec = make_uint2(0u, 0u);
			if (ne > 0) {
				int m, fwd, bwd;
				if (le - fe + 1 == ne) {
					int lo = 0, hi = (int)nn - 1;
					for (;;) {
						m = (lo + hi) >> 1;
						if (m < fe) lo = m + 1;
						else if (m > le) hi = m - 1;
						else break;
					}
					fwd = le - m + 1;
					bwd = m - fe;
				} else {
					const int16_t kq = (int16_t)k16;
					bool hit = false;
					int lo = 0, hi = (int)nn - 1;
					m = 0;
					for (;;) {
						m = (lo + hi) >> 1;
						const int16_t kk = K[m];
						if (kk > kq) hi = m - 1;
						else if (kk < kq) lo = m + 1;
						else { hit = true; break; }
						if (hi < lo) break;
					}
					fwd = bwd = 0;
					if (hit) {
						int qq = m + 1;
						while (qq < (int)nn && K[qq] == kq) qq++;
						fwd = qq - m;
						qq = m - 1;
						while (qq >= 0 && K[qq] == kq) qq--;
						bwd = m - 1 - qq;
					}
				}
				if (fwd + bwd > 0) rec = make_uint2(first + (uint32_t)m, (uint32_t)fwd | ((uint32_t)bwd << 16));
			}
			if (sub == 0) {
				pp.out[outidx] = rec;
				st_i += nn;
				st_h += (rec.y & 0xffffu) + (rec.y >> 16);
			}
		}
	}
	if (pp.stats) {
		for (int o = 32; o; o >>= 1) {
			st_i += __shfl_xor(st_i, o); st_h += __shfl_xor(st_h, o); st_n += __shfl_xor(st_n, o);
		}
		if (lane_id() == 0 && (st_i || st_h || st_n)) {
			atomicAdd(&pp.stats[1], st_i);
			atomicAdd(&pp.stats[2], st_h);
			atomicAdd(&pp.stats[5], st_n);   // diagnostics: probes searched here
		}
	}
}

// =============================================================================================
// host side: handle, upload, launch
// =============================================================================================

// compact probe images (DevIndex::bgrp, keys8)
__global__ void __launch_bounds__(256) build_bgrp(const uint32_t *bstart, uint32_t nb, uint32_t *bgrp)
{
	const uint32_t ng = (nb + 15) / 16;
	for (uint32_t g = blockIdx.x * 256u + threadIdx.x; g < ng; g += gridDim.x * 256u) {
		uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
		w[0] = bstart[16 * g];
#pragma unroll
		for (int i = 0; i < 16; i++) {
			const uint32_t b = 16 * g + (uint32_t)i;
			uint32_t c = 0;
			if (b < nb) { c = bstart[b + 1] - bstart[b]; if (c > 255) c = 255; }
			w[1 + (i >> 2)] |= c << (8 * (i & 3));
		}
		uint4 *d = (uint4 *)(bgrp + 8 * (size_t)g);
		d[0] = make_uint4(w[0], w[1], w[2], w[3]);
		d[1] = make_uint4(w[4], w[5], w[6], w[7]);
	}
}

__global__ void __launch_bounds__(256) build_keys8(const int16_t *keys, uint64_t items, uint8_t *keys8)
{
	for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < items; i += (uint64_t)gridDim.x * 256u)
		keys8[i] = (uint8_t)keys[i];
}

// DevIndex::bcode: one 32-byte sector per bucket -- u32 first item, u8 item count (255 = not coded:
// more than 216 - V items, or keys not sorted), then the bucket's sorted key_hi multiset as a
// unary count code over bits 40..255: for v = 0 .. V-1, c_v one-bits then a zero (V = number of
// possible key_hi values, key / nb <= 0xffffffff / nb; 47 at nb = 93,018,839), rest one-bits.
// The equal-key run of key_hi k is then [ones before zero k-1, ones before zero k): a probe needs
// one random 32-byte sector instead of a 64-byte line (HBM serves ~1.6x more of them per second).
#define BCODE_BITS 216
__global__ void __launch_bounds__(256) build_bcode(const uint32_t *bstart, const int16_t *keys, uint32_t nb, int V, uint4 *bcode)
{
	for (uint32_t b = blockIdx.x * 256u + threadIdx.x; b < nb; b += gridDim.x * 256u) {
		const uint32_t first = bstart[b], n = bstart[b + 1] - first;
		uint32_t w[8];
#pragma unroll
		for (int q = 0; q < 8; q++) w[q] = 0xffffffffu;   // unused tail: one-bits
		w[0] = first;
		bool ok = (int)n + V <= BCODE_BITS;
		if (ok) {
			int pos = 40, cur = 0;
			for (uint32_t i = 0; i < n && ok; i++) {
				const int v = keys[first + i];
				if (v < cur || v >= V) { ok = false; break; }
				while (cur < v) { w[pos >> 5] &= ~(1u << (pos & 31)); pos++; cur++; }   // zero: value cur closed
				pos++;                                                            // one: an item of value v
			}
			while (ok && cur < V) { w[pos >> 5] &= ~(1u << (pos & 31)); pos++; cur++; }
		}
		w[1] = (w[1] & 0xffffff00u) | (ok ? n : 255u);
		uint4 *d = bcode + 2 * (size_t)b;
		d[0] = make_uint4(w[0], w[1], w[2], w[3]);
		d[1] = make_uint4(w[4], w[5], w[6], w[7]);
	}
}

// the payload words of every line start at 0 (the keys at 0xffffffff: empty)
template <bool SEC>
__global__ void __launch_bounds__(256) clear_khash_payload(uint32_t *kh, uint64_t lines)
{
	for (uint64_t L = blockIdx.x * 256ull + threadIdx.x; L < lines; L += gridDim.x * 256ull) {
		if (SEC) { uint32_t *w = kh + 8 * L; w[3] = w[4] = w[5] = w[6] = w[7] = 0u; }
		else kh[16 * L + 15] = 0u;
	}
}

// DevIndex::khash: for every distinct key of every bucket, gehash_go_X's binary search
// (sorted-hashtable.c:947-981) run here once -- first hit midpoint m, equal keys after / before
// it -- and the resulting probe record stored under the full key.  A probe then costs one random
// sector (SEC: 32 bytes, 3 entries with 8-bit run counts) or line (64 bytes, 5 entries) whatever
// the bucket's size (gapped indexes: ~87 items per bucket at 3 Gbp).  ff[3] is set when a run
// count does not fit 8 bits (the sector image is then not used).
template <bool SEC>
__global__ void __launch_bounds__(256) build_khash(const uint32_t *bstart, const int16_t *keys, uint32_t nb, uint32_t *kh,
                                                   uint64_t lines, uint32_t *ff)
{
	for (uint32_t b = blockIdx.x * 256u + threadIdx.x; b < nb; b += gridDim.x * 256u) {
		const uint32_t first = bstart[b], n = bstart[b + 1] - first;
		const int16_t *K = keys + first;
		for (uint32_t j = 0; j < n; j++) {
			const int16_t k16 = K[j];
			if (j > 0 && K[j - 1] == k16) continue;   // the run's first item (a repeated run inserts once)
			int lo = 0, hi = (int)n - 1, m = 0;
			bool hit = false;
			for (;;) {
				m = (lo + hi) >> 1;
				const int16_t kk = K[m];
				if (kk > k16) hi = m - 1;
				else if (kk < k16) lo = m + 1;
				else { hit = true; break; }
				if (hi < lo) break;
			}
			if (!hit) continue;   // an unsorted bucket can hide a key from the search: no record
			int qq = m + 1;
			while (qq < (int)n && K[qq] == k16) qq++;
			const uint32_t fwd = (uint32_t)(qq - m);
			qq = m - 1;
			while (qq >= 0 && K[qq] == k16) qq--;
			const uint32_t bwd = (uint32_t)(m - 1 - qq);
			const uint32_t key = (uint32_t)(uint16_t)k16 * nb + b, ry = fwd | (bwd << 16);
			const uint32_t rx = first + (uint32_t)m;
			if (key == 0xffffffffu) { ff[1] = rx; ff[2] = ry; ff[0] = 1u; continue; }
			if (SEC && (fwd > 255u || bwd > 255u)) { atomicOr(&ff[3], 1u); continue; }
			uint64_t L = khash_line(key, lines);
			for (;;) {
				uint32_t *w = kh + (SEC ? 8 : 16) * L;
				const int slots = SEC ? 3 : 5;
				int s = 0;
				for (; s < slots; s++) {
					const uint32_t old = atomicCAS(&w[s], 0xffffffffu, key);
					if (old == 0xffffffffu) {
						if (SEC) {
							w[3 + s] = rx;
							atomicOr(&w[6 + (s >> 1)], (fwd | (bwd << 8)) << (16 * (s & 1)));
						} else {
							w[5 + 2 * s] = rx;
							w[6 + 2 * s] = ry;
						}
						break;
					}
					if (old == key) break;
				}
				if (s < slots) break;
				atomicOr(SEC ? &w[7] : &w[15], SEC ? 1u << 16 : 1u);   // full: lookups continue at the next line
				L = L + 1 == lines ? 0 : L + 1;
			}
		}
	}
}

// DevIndex::ksorted: one bit per bucket, set when the bucket's keys are non-decreasing as shorts
__global__ void __launch_bounds__(256) build_ksorted(const uint32_t *bstart, const int16_t *keys, uint32_t nb, uint32_t *bits)
{
	const uint32_t nw = (nb + 31) / 32;
	for (uint32_t w = blockIdx.x * 256u + threadIdx.x; w < nw; w += gridDim.x * 256u) {
		uint32_t m = 0;
		for (uint32_t k = 0; k < 32; k++) {
			const uint32_t b = w * 32 + k;
			if (b >= nb) break;
			const uint32_t first = bstart[b], n = bstart[b + 1] - first;
			bool ok = true;
			for (uint32_t j = 1; j < n && ok; j++) ok = keys[first + j - 1] <= keys[first + j];
			m |= (ok ? 1u : 0u) << k;
		}
		bits[w] = m;
	}
}

// DevIndex::bline: one 64-byte line per bucket (first item, count, the u8 keys of <= 59 items)
__global__ void __launch_bounds__(256) build_bline(const uint32_t *bstart, const int16_t *keys, uint32_t nb, uint4 *bline)
{
	for (uint32_t b = blockIdx.x * 256u + threadIdx.x; b < nb; b += gridDim.x * 256u) {
		const uint32_t first = bstart[b], n = bstart[b + 1] - first;
		uint32_t w[16];
#pragma unroll
		for (int q = 0; q < 16; q++) w[q] = 0u;
		w[0] = first;
		w[1] = n > 255u ? 255u : n;
		if (n <= 59u) {
#pragma unroll
			for (int i = 0; i < 59; i++)
				if ((uint32_t)i < n) w[(5 + i) >> 2] |= (uint32_t)(uint8_t)keys[first + i] << (8 * ((5 + i) & 3));
		}
		uint4 *d = bline + 4 * (size_t)b;
#pragma unroll
		for (int q = 0; q < 4; q++) d[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
	}
}

// The library's four streams of a device (probe + lane kernels, wave kernel + compaction, uploads,
// downloads) are one set per process, created back to back and shared by every handle on the
// device.  HIP deals a process's streams round-robin onto GPU_MAX_HW_QUEUES (4) hardware queues:
// four consecutive creations land on four different queues, whereas per-handle streams created at
// different times (a second index, a multi-block index's blocks, torch's own streams in between)
// can put a handle's two kernel streams on one queue, where the wave kernel of chunk c and the
// probe kernel of chunk c+1 run one after the other -- measured in a three-index process:
// 152 ms/step against 110 with the same kernels (profiles/r04/ab_images_c3.json).  Handles on one
// device then order their work on the same streams, which changes no result (each handle's
// buffers are its own; its calls already wait for its previous call).
static pthread_mutex_t g_streams_mu = PTHREAD_MUTEX_INITIALIZER;
static struct { hipStream_t s[4]; int refs; } g_streams[64];

static int streams_acquire(svg_index *h)
{
	if (h->device < 0 || h->device >= 64) { svg_set_error("device %d out of range", h->device); return SVG_E_ARG; }
	pthread_mutex_lock(&g_streams_mu);
	int rc = 0;
	if (!g_streams[h->device].refs) {
		// (round 4 measured CU-masked streams for the wave kernel: 64 / 96 / 128 / 192 of 256 CUs
		// gave 219.8 / 162.4 / 144.5 / 101.7 ms/step against 100.7 unmasked)
		for (int k = 0; k < 4 && !rc; k++) {
			const hipError_t e = hipStreamCreateWithFlags(&g_streams[h->device].s[k], hipStreamNonBlocking);
			if (e != hipSuccess) {
				svg_set_error("hipStreamCreate failed");
				rc = SVG_E_DEVICE;
				for (int j = 0; j < k; j++) hipStreamDestroy(g_streams[h->device].s[j]);
			}
		}
	}
	if (!rc) {
		g_streams[h->device].refs++;
		h->stream = g_streams[h->device].s[0];
		h->stream2 = g_streams[h->device].s[1];
		h->up_stream = g_streams[h->device].s[2];
		h->down_stream = g_streams[h->device].s[3];
	}
	pthread_mutex_unlock(&g_streams_mu);
	return rc;
}

static void streams_release(svg_index *h)
{
	if (!h->stream) return;
	pthread_mutex_lock(&g_streams_mu);
	if (--g_streams[h->device].refs == 0)
		for (int k = 0; k < 4; k++) hipStreamDestroy(g_streams[h->device].s[k]);
	pthread_mutex_unlock(&g_streams_mu);
	h->stream = h->stream2 = h->up_stream = h->down_stream = NULL;
}

// common tail of svg_index_open / svg_index_build*: d_bstart/d_keys/d_vals already in HBM,
// host part holds .array and the chromosome table
int svg_index_finish_device(svg_index *h)
{
	svg_host_index *x = &h->host;
	int rc;
	h->nblocks = 1;
	HIPCHK(hipSetDevice(h->device));
	if ((rc = dmalloc(h, &h->d_values, (size_t)x->values_bytes + 64)) || (rc = dmalloc(h, &h->d_chr, 4 * (size_t)x->n_chr + 64)))
		return rc;
	if ((rc = streams_acquire(h))) return rc;
	HIPCHK(hipEventCreateWithFlags(&h->ev_up[2], hipEventDisableTiming));
	HIPCHK(hipEventCreateWithFlags(&h->ev_done[2], hipEventDisableTiming));
	HIPCHK(hipEventCreateWithFlags(&h->ev_down[2], hipEventDisableTiming));
	for (int s = 0; s < 3; s++) {
		HIPCHK(hipEventCreateWithFlags(&h->ev_lane[s], hipEventDisableTiming));
		HIPCHK(hipEventCreateWithFlags(&h->ev_wave[s], hipEventDisableTiming));
		HIPCHK(hipEventCreateWithFlags(&h->ev_probe[s], hipEventDisableTiming));
	}
	for (int s = 0; s < 2; s++) {
		HIPCHK(hipEventCreateWithFlags(&h->ev_up[s], hipEventDisableTiming));
		HIPCHK(hipEventCreateWithFlags(&h->ev_done[s], hipEventDisableTiming));
		HIPCHK(hipEventCreateWithFlags(&h->ev_down[s], hipEventDisableTiming));
	}
	HIPCHK(hipMemcpy(h->d_values, x->values, x->values_bytes, hipMemcpyHostToDevice));
	HIPCHK(hipMemcpy(h->d_chr, x->chr_end, 4 * (size_t)x->n_chr, hipMemcpyHostToDevice));
	h->dix.bstart = (const uint32_t *)h->d_bstart;
	h->dix.keys = (const int16_t *)h->d_keys;
	h->dix.vals = (const uint32_t *)h->d_vals;
	h->dix.values = (const uint8_t *)h->d_values;
	h->dix.chr_end = (const uint32_t *)h->d_chr;
	h->dix.nb = x->nb;
	h->dix.n_chr = x->n_chr;
	h->dix.start_point = x->start_point;
	h->dix.length = x->length;
	h->dix.start_base_offset = x->start_base_offset;
	h->dix.values_bytes = x->values_bytes;
	h->dix.gap = x->gap;
	h->dix.padding = x->padding;
	hipDeviceProp_t prop;
	HIPCHK(hipGetDeviceProperties(&prop, h->device));
	h->n_cu = prop.multiProcessorCount;
	h->dix.bgrp = NULL;
	h->dix.keys8 = NULL;
	h->dix.bline = NULL;
	h->dix.bcode = NULL;
	h->dix.khash = NULL;
	h->dix.khash_ff = NULL;
	h->dix.khash_lines = 0;
	h->dix.khash_sec = 0;
	h->dix.ksorted = NULL;
	{
		// 32-byte bucket codes when the key_hi range is small enough for them to hold ordinary
		// buckets (V = 47 at nb = 93,018,839, the -F -B full index): n + V <= 216 bits
		const uint32_t V = 0xffffffffu / x->nb + 1u;
		if (V <= 80u && !svg_get_option("no_compact") && !svg_get_option("no_bcode")) {
			if (dmalloc(h, &h->d_bcode, (size_t)x->nb * 32 + 64) == 0) {
				uint64_t blocks = ((uint64_t)x->nb + 255) / 256, bmax = (uint64_t)h->n_cu * 64;
				if (blocks > bmax) blocks = bmax;
				hipLaunchKernelGGL(build_bcode, dim3((unsigned)blocks), dim3(256), 0, h->stream, (const uint32_t *)h->d_bstart,
				                   (const int16_t *)h->d_keys, x->nb, (int)V, (uint4 *)h->d_bcode);
				HIPCHK(hipGetLastError());
				HIPCHK(hipStreamSynchronize(h->stream));
				h->dix.bcode = (const uint4 *)h->d_bcode;
			} else {
				h->d_bcode = NULL;
				(void)hipGetLastError();
			}
		}
	}
	// the key-hash image: the probe image of indexes the bucket code does not fit (gapped, small);
	// beside the code it was measured at C3 (profiles/r04/bench_c3_*.json): the key-hash probe
	// kernel is 18% faster than the code's, but the lane / wave kernels slow by more than that
	// (113.5 vs 110.6 ms/step), so the code is the probe image of -F -B indexes.  The code, when it fits, also serves the paths that need
	// item indices (svg_probe_keys, fragile and sublong voting).  (Round 4 also measured the key-hash
	// image beside the code with one-hit runs inline -- the hit's position in the probe record, no
	// vals[] load -- 52 GB at C3, slower: 113.5 vs 110.6 ms/step; removed.)
	if (!h->dix.bcode && !svg_get_option("no_compact") && !svg_get_option("no_khash")) {
		// key-hash image of the probe records: 32-byte sectors of 3 entries (lines ~ items / 1.8),
		// or 64-byte lines of 5 entries (~ items / 3) when a run count needs more than 8 bits
		for (int sec = svg_get_option("khash64") ? 0 : 1; sec >= 0 && !h->dix.khash; sec--) {
			const uint64_t lines = (sec ? x->items * 5 / 9 : x->items / 3) + 1024, lb = sec ? 32 : 64;
			if (dmalloc(h, &h->d_khash, lines * lb + 64) != 0) {
				h->d_khash = NULL;
				(void)hipGetLastError();
				break;
			}
			uint32_t *ff = (uint32_t *)((uint8_t *)h->d_khash + lines * lb);
			HIPCHK(hipMemsetAsync(h->d_khash, 0xff, lines * lb, h->stream));
			HIPCHK(hipMemsetAsync(ff, 0, 64, h->stream));
			uint64_t blocks = (lines + 255) / 256, bmax = (uint64_t)h->n_cu * 64;
			if (blocks > bmax) blocks = bmax;
			if (sec) hipLaunchKernelGGL(clear_khash_payload<true>, dim3((unsigned)blocks), dim3(256), 0, h->stream, (uint32_t *)h->d_khash, lines);
			else hipLaunchKernelGGL(clear_khash_payload<false>, dim3((unsigned)blocks), dim3(256), 0, h->stream, (uint32_t *)h->d_khash, lines);
			HIPCHK(hipGetLastError());
			blocks = ((uint64_t)x->nb + 255) / 256;
			if (blocks > bmax) blocks = bmax;
			if (sec)
				hipLaunchKernelGGL(build_khash<true>, dim3((unsigned)blocks), dim3(256), 0, h->stream, (const uint32_t *)h->d_bstart,
				                   (const int16_t *)h->d_keys, x->nb, (uint32_t *)h->d_khash, lines, ff);
			else
				hipLaunchKernelGGL(build_khash<false>, dim3((unsigned)blocks), dim3(256), 0, h->stream, (const uint32_t *)h->d_bstart,
				                   (const int16_t *)h->d_keys, x->nb, (uint32_t *)h->d_khash, lines, ff);
			HIPCHK(hipGetLastError());
			uint32_t wide = 0;
			HIPCHK(hipMemcpyAsync(&wide, ff + 3, 4, hipMemcpyDeviceToHost, h->stream));
			HIPCHK(hipStreamSynchronize(h->stream));
			if (sec && wide) {   // a run of more than 255 equal keys (repeat threshold > 255): 64-byte lines
				h->device_bytes -= lines * lb + 64;
				HIPCHK(hipFree(h->d_khash));
				h->d_khash = NULL;
				continue;
			}
			h->dix.khash = (const uint32_t *)h->d_khash;
			h->dix.khash_ff = ff;
			h->dix.khash_lines = lines;
			h->dix.khash_sec = sec;
		}
		// which buckets are sorted: there the key-hash record is cellCounts' equal-key run too
		if (h->dix.khash && dmalloc(h, &h->d_ksorted, ((size_t)x->nb + 31) / 32 * 4 + 64) == 0) {
			uint64_t blocks = ((uint64_t)x->nb / 32 + 256) / 256, bmax = (uint64_t)h->n_cu * 64;
			if (blocks > bmax) blocks = bmax;
			hipLaunchKernelGGL(build_ksorted, dim3((unsigned)blocks), dim3(256), 0, h->stream, (const uint32_t *)h->d_bstart,
			                   (const int16_t *)h->d_keys, x->nb, (uint32_t *)h->d_ksorted);
			HIPCHK(hipGetLastError());
			HIPCHK(hipStreamSynchronize(h->stream));
			h->dix.ksorted = (const uint32_t *)h->d_ksorted;
		} else if (h->dix.khash) {
			h->d_ksorted = NULL;
			(void)hipGetLastError();
		}
	}
	if (!h->dix.bcode && !h->dix.khash && x->nb >= 16843009u && !svg_get_option("no_compact") && !svg_get_option("no_bline")) {
		// (2^32-1)/nb <= 255: every key_hi fits a byte; 64 B per bucket (5.95 GB at nb = 93M)
		// optional image: without the HBM for it the index still opens with the group/key images
		if (dmalloc(h, &h->d_bline, (size_t)x->nb * 64 + 64) == 0) {
			uint64_t blocks = ((uint64_t)x->nb + 255) / 256, bmax = (uint64_t)h->n_cu * 64;
			if (blocks > bmax) blocks = bmax;
			hipLaunchKernelGGL(build_bline, dim3((unsigned)blocks), dim3(256), 0, h->stream, (const uint32_t *)h->d_bstart,
			                   (const int16_t *)h->d_keys, x->nb, (uint4 *)h->d_bline);
			HIPCHK(hipGetLastError());
			HIPCHK(hipStreamSynchronize(h->stream));
			h->dix.bline = (const uint4 *)h->d_bline;
		} else {
			h->d_bline = NULL;
			(void)hipGetLastError();
		}
	}
	if (!h->dix.bline && !h->dix.bcode && !h->dix.khash && x->nb >= 16843009u && !svg_get_option("no_compact")) {
		// (2^32-1)/nb <= 255: every key_hi fits a byte
		const size_t ng = ((size_t)x->nb + 15) / 16;
		if ((rc = dmalloc(h, &h->d_bgrp, ng * 32 + 64)) || (rc = dmalloc(h, &h->d_keys8, x->items + 128))) return rc;
		uint64_t blocks = (ng + 255) / 256, bmax = (uint64_t)h->n_cu * 64;
		if (blocks > bmax) blocks = bmax;
		hipLaunchKernelGGL(build_bgrp, dim3((unsigned)blocks), dim3(256), 0, h->stream, (const uint32_t *)h->d_bstart, x->nb,
		                   (uint32_t *)h->d_bgrp);
		HIPCHK(hipGetLastError());
		blocks = (x->items + 255) / 256;
		if (blocks > bmax) blocks = bmax;
		hipLaunchKernelGGL(build_keys8, dim3((unsigned)blocks), dim3(256), 0, h->stream, (const int16_t *)h->d_keys, x->items,
		                   (uint8_t *)h->d_keys8);
		HIPCHK(hipGetLastError());
		HIPCHK(hipMemsetAsync((uint8_t *)h->d_keys8 + x->items, 0, 128, h->stream));
		HIPCHK(hipStreamSynchronize(h->stream));
		h->dix.bgrp = (const uint32_t *)h->d_bgrp;
		h->dix.keys8 = (const uint8_t *)h->d_keys8;
	}
	if ((rc = dmalloc(h, (void **)&h->d_stats, 32 * sizeof(unsigned long long)))) return rc;
	HIPCHK(hipMemset(h->d_stats, 0, 32 * sizeof(unsigned long long)));
	if ((rc = dmalloc(h, (void **)&h->d_err, 64))) return rc;
	HIPCHK(hipMemset(h->d_err, 0, 64));
	HIPCHK(hipEventCreateWithFlags(&h->ev_last, hipEventDisableTiming));
	h->stats_on = 0;
	h->max_read_len = 256;
	return 0;
}

// One block from its files into HBM.  The .tab is a chain of bucket records {i32 n, i32 space,
// i16 keys[n], u32 vals[n]}: where bucket b + 1 starts is known only from bucket b's n, and a
// serial walk of the chain is one dependent memory load per bucket (C3: 93M buckets, 11.7 s).
// The walk is split instead: worker t finds, from byte S_t = t/T of the file on, the first offset
// where a run of WALK_SYNC consecutive records is well formed (n == space -- what gehash_dump and
// our builder write, sorted-hashtable.c:1867-1870 --, sizes inside the file) and walks the chain
// from there; worker t's walk must land exactly on worker t+1's start (the last one on the file's
// final byte), which proves every start right -- otherwise one serial walk is done instead.
// Then bucket starts are a prefix sum, and the workers gather runs of buckets (~LOAD_ITEMS items)
// from the mapped file into pinned staging buffers and copy them to d_keys / d_vals on streams of
// their own; the .array and .reads load beside them.  No host copy of the 21 GB arrays is made
// (round 4 read them into malloc'd arrays, then uploaded pageable memory: 19.1 s at C3).
#define LOAD_ITEMS (4u << 20)
#define LOAD_WORKERS 16
#define LOAD_BUFS 2
#define WALK_SYNC 32

// a well-formed run of WALK_SYNC records from p (the file's buckets end at `last`)
static bool tab_sync_ok(const uint8_t *p, const uint8_t *last)
{
	for (int k = 0; k < WALK_SYNC; k++) {
		if (p == last) return k > 0;
		if (p + 8 > last) return false;
		int32_t n, sp;
		memcpy(&n, p, 4);
		memcpy(&sp, p + 4, 4);
		if (n < 0 || n != sp || (uint64_t)(last - p) < 8 + 6 * (uint64_t)(uint32_t)n) return false;
		p += 8 + 6 * (size_t)(uint32_t)n;
	}
	return true;
}

// the bucket sizes of the chain from `first` to `last`, in order; false: not a chain of nb buckets
static bool tab_walk(const uint8_t *first, const uint8_t *last, uint32_t nb, uint32_t *sizes, int nt)
{
	const uint64_t len = (uint64_t)(last - first);
	std::vector<const uint8_t *> start(nt + 1, NULL);
	std::vector<std::vector<uint32_t>> part(nt);
	std::vector<const uint8_t *> stop(nt, NULL);
	start[0] = first;
	start[nt] = last;
	// starts: candidate offsets keep first's parity (every record is an even number of bytes)
	{
		std::vector<std::thread> th;
		for (int t = 1; t < nt; t++)
			th.emplace_back([&, t] {
				const uint8_t *q = first + len * (uint64_t)t / (uint64_t)nt;
				if ((q - first) & 1) q++;
				const uint8_t *lim = first + len * (uint64_t)(t + 1) / (uint64_t)nt;
				for (; q < lim; q += 2)
					if (tab_sync_ok(q, last)) { start[t] = q; return; }
			});
		for (auto &x : th) x.join();
	}
	// segments without a start merge into the one before them
	std::vector<int> seg;
	for (int t = 0; t < nt; t++) if (start[t]) seg.push_back(t);
	const int ns = (int)seg.size();
	std::vector<const uint8_t *> s0(ns + 1);
	for (int k = 0; k < ns; k++) s0[k] = start[seg[k]];
	s0[ns] = last;
	{
		std::vector<std::thread> th;
		for (int k = 0; k < ns; k++)
			th.emplace_back([&, k] {
				const uint8_t *p = s0[k], *until = s0[k + 1];
				std::vector<uint32_t> &v = part[k];
				v.reserve((size_t)((until - p) / 150 + 16));
				while (p < until) {
					if (p + 8 > last) break;
					int32_t n;
					memcpy(&n, p, 4);
					if (n < 0 || (uint64_t)(last - p) < 8 + 6 * (uint64_t)(uint32_t)n) break;
					v.push_back((uint32_t)n);
					p += 8 + 6 * (size_t)(uint32_t)n;
				}
				stop[k] = p;
			});
		for (auto &x : th) x.join();
	}
	bool ok = true;
	uint64_t total = 0;
	for (int k = 0; k < ns; k++) {
		if (stop[k] != s0[k + 1]) ok = false;
		total += part[k].size();
	}
	if (ok && total == nb) {
		uint64_t b = 0;
		for (int k = 0; k < ns; k++) {
			memcpy(sizes + b, part[k].data(), 4 * part[k].size());
			b += part[k].size();
		}
		return true;
	}
	// one serial walk
	const uint8_t *p = first;
	for (uint32_t b = 0; b < nb; b++) {
		if (p + 8 > last) return false;
		int32_t n;
		memcpy(&n, p, 4);
		if (n < 0 || (uint64_t)(last - p) < 8 + 6 * (uint64_t)(uint32_t)n) return false;
		sizes[b] = (uint32_t)n;
		p += 8 + 6 * (size_t)(uint32_t)n;
	}
	return p == last;
}

// a second handle's copy of the host side of block `src` (the .array image, contig table, counts)
static int host_meta_copy(const svg_host_index *src, svg_host_index *dst)
{
	*dst = *src;
	dst->map = NULL;
	dst->map_len = 0;
	dst->bstart = NULL;
	dst->keys = NULL;
	dst->vals = NULL;
	dst->values = NULL;
	dst->chr_end = NULL;
	dst->chr_name = NULL;
	if (src->values && !(dst->values = (uint8_t *)malloc((size_t)src->values_bytes + 8))) return SVG_E_NOMEM;
	if (src->values) memcpy(dst->values, src->values, (size_t)src->values_bytes + 8);
	if (src->n_chr) {
		dst->chr_end = (uint32_t *)malloc(4 * (size_t)src->n_chr);
		dst->chr_name = (char (*)[200])malloc(200 * (size_t)src->n_chr);
		if (!dst->chr_end || !dst->chr_name) return SVG_E_NOMEM;
		memcpy(dst->chr_end, src->chr_end, 4 * (size_t)src->n_chr);
		memcpy(dst->chr_name, src->chr_name, 200 * (size_t)src->n_chr);
	}
	return 0;
}

// One block of the index into HBM of every device in devs[0..n-1] (one handle each; a device may
// repeat): the .tab is mapped, walked and gathered into pinned staging runs ONCE, and every run is
// copied to every handle's arrays (one stream per worker and handle); the .array and contig table
// are read once and copied to each handle; each handle then builds its device images on a thread of
// its own.  n = 1 is svg_index_open's single replica.
static int index_open_block_multi(const char *prefix, int block, const int *devs, int n, svg_index **outs)
{
	for (int k = 0; k < n; k++) outs[k] = NULL;
	std::vector<svg_index *> h(n, (svg_index *)NULL);
	auto drop_all = [&]() { for (int k = 0; k < n; k++) if (h[k]) { svg_index_close(h[k]); h[k] = NULL; } };
	for (int k = 0; k < n; k++) {
		if (!(h[k] = (svg_index *)calloc(1, sizeof(svg_index)))) { drop_all(); svg_set_error("out of memory"); return SVG_E_NOMEM; }
		h[k]->device = devs[k];
		h[k]->nblocks = 1;
	}
	const bool dbg = (svg_get_option("debug") & 8) != 0;
	auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
	const double t0 = now();
	svg_host_index *x = &h[0]->host;
	char fn[4096];
	snprintf(fn, sizeof fn, "%s.%02d.b.tab", prefix, block);
	const uint8_t *first = NULL;
	int rc = svg_tab_map(fn, x, &first);
	if (rc) { drop_all(); return rc; }
	// the .array and the contig table on a thread of their own
	// (svg_set_error's buffer is per thread: a failure's message comes back with meta_rc)
	int meta_rc = 0;
	char meta_err[256] = "";
	std::thread meta([&] {
		meta_rc = svg_host_index_load_meta(prefix, block, x);
		if (meta_rc) snprintf(meta_err, sizeof meta_err, "%s", svg_last_error());
	});
	// the buckets end one byte before the file does (gehash_dump's is_small_table byte)
	const uint8_t *const last = (const uint8_t *)x->map + x->map_len - 1;
	uint32_t *bstart = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)x->nb + 1));
	if (!bstart) { rc = SVG_E_NOMEM; svg_set_error("out of memory"); }
	for (int k = 0; k < n && !rc; k++) {
		if (hipSetDevice(devs[k]) != hipSuccess) { rc = SVG_E_DEVICE; svg_set_error("hipSetDevice(%d) failed", devs[k]); break; }
		if ((rc = dmalloc(h[k], &h[k]->d_bstart, 4 * ((size_t)x->nb + 1))) || (rc = dmalloc(h[k], &h[k]->d_keys, 2 * x->items + 64)) ||
		    (rc = dmalloc(h[k], &h[k]->d_vals, 4 * x->items + 64)))
			break;
	}
	double t_walk = 0, t_copy = 0;
	if (!rc) {
		if (!tab_walk(first, last, x->nb, bstart, LOAD_WORKERS)) {
			rc = SVG_E_FORMAT;
			svg_set_error("'%s': the bucket records do not make %u buckets", fn, x->nb);
		} else {
			uint64_t cur = 0;
			for (uint32_t b = 0; b < x->nb; b++) {
				const uint32_t c = bstart[b];
				bstart[b] = (uint32_t)cur;
				cur += c;
			}
			bstart[x->nb] = (uint32_t)cur;
			if (cur != x->items) { rc = SVG_E_FORMAT; svg_set_error("'%s': bucket sizes do not add up", fn); }
		}
		t_walk = now() - t0;
	}
	if (!rc) {
		// runs of buckets [b0, b1) of at most LOAD_ITEMS items (a staging buffer), or a single
		// bucket larger than that (copied straight from the map below)
		std::vector<std::pair<uint32_t, uint32_t>> jobs;
		{
			uint32_t b0 = 0;
			for (uint32_t b = 0; b < x->nb; b++)
				if (b > b0 && (uint64_t)bstart[b + 1] - bstart[b0] > LOAD_ITEMS) {
					jobs.emplace_back(b0, b);
					b0 = b;
				}
			if (b0 < x->nb) jobs.emplace_back(b0, x->nb);
		}
		std::atomic<size_t> next(0);
		std::atomic<int> werr(0);
		auto worker = [&]() {
			std::vector<hipStream_t> st(n, (hipStream_t)NULL);
			uint8_t *buf[LOAD_BUFS] = {NULL, NULL};
			std::vector<hipEvent_t> ev((size_t)LOAD_BUFS * n, (hipEvent_t)NULL);
			bool used[LOAD_BUFS] = {false, false};
			int kb_ = 0;
			for (int k = 0; k < n && !werr; k++) {
				if (hipSetDevice(devs[k]) != hipSuccess || hipStreamCreateWithFlags(&st[k], hipStreamNonBlocking) != hipSuccess) werr = 1;
				for (int i = 0; i < LOAD_BUFS && !werr; i++)
					if (hipEventCreateWithFlags(&ev[i * n + k], hipEventDisableTiming) != hipSuccess) werr = 1;
			}
			for (int i = 0; i < LOAD_BUFS && !werr; i++)
				if (hipHostMalloc((void **)&buf[i], 6 * (size_t)LOAD_ITEMS, hipHostMallocDefault | hipHostMallocPortable) != hipSuccess) werr = 1;
			for (;;) {
				const size_t jn = next.fetch_add(1);
				if (jn >= jobs.size() || werr) break;
				const uint32_t b0 = jobs[jn].first, b1 = jobs[jn].second;
				const uint64_t i0 = bstart[b0], cnt = (uint64_t)bstart[b1] - i0;
				if (!cnt) continue;
				if (cnt > LOAD_ITEMS) {   // one bucket larger than a staging buffer (b1 == b0 + 1): straight from the map
					const uint8_t *src = first + 8ull * b0 + 6ull * i0 + 8;
					for (int k = 0; k < n && !werr; k++)
						if (hipSetDevice(devs[k]) != hipSuccess ||
						    hipMemcpy((uint8_t *)h[k]->d_keys + 2 * i0, src, 2 * cnt, hipMemcpyHostToDevice) != hipSuccess ||
						    hipMemcpy((uint8_t *)h[k]->d_vals + 4 * i0, src + 2 * cnt, 4 * cnt, hipMemcpyHostToDevice) != hipSuccess)
							werr = 1;
					continue;
				}
				if (used[kb_])
					for (int k = 0; k < n; k++)
						if (hipEventSynchronize(ev[kb_ * n + k]) != hipSuccess) werr = 1;
				if (werr) break;
				uint8_t *kb = buf[kb_], *vb = buf[kb_] + 2 * (size_t)LOAD_ITEMS;
				for (uint32_t b = b0; b < b1; b++) {
					const uint64_t c = (uint64_t)bstart[b + 1] - bstart[b], at = (uint64_t)bstart[b] - i0;
					if (!c) continue;
					const uint8_t *src = first + 8ull * b + 6ull * bstart[b] + 8;
					memcpy(kb + 2 * at, src, 2 * c);
					memcpy(vb + 4 * at, src + 2 * c, 4 * c);
				}
				for (int k = 0; k < n && !werr; k++)
					if (hipSetDevice(devs[k]) != hipSuccess ||
					    hipMemcpyAsync((uint8_t *)h[k]->d_keys + 2 * i0, kb, 2 * cnt, hipMemcpyHostToDevice, st[k]) != hipSuccess ||
					    hipMemcpyAsync((uint8_t *)h[k]->d_vals + 4 * i0, vb, 4 * cnt, hipMemcpyHostToDevice, st[k]) != hipSuccess ||
					    hipEventRecord(ev[kb_ * n + k], st[k]) != hipSuccess)
						werr = 1;
				used[kb_] = true;
				kb_ = (kb_ + 1) % LOAD_BUFS;
			}
			for (int k = 0; k < n; k++)
				if (st[k]) {
					hipSetDevice(devs[k]);
					if (hipStreamSynchronize(st[k]) != hipSuccess) werr = 1;
					hipStreamDestroy(st[k]);
				}
			for (auto e : ev)
				if (e) hipEventDestroy(e);
			for (int i = 0; i < LOAD_BUFS; i++)
				if (buf[i]) hipHostFree(buf[i]);
		};
		std::vector<std::thread> ws;
		for (int t = 0; t < LOAD_WORKERS; t++) ws.emplace_back(worker);
		for (auto &w : ws) w.join();
		if (werr) { rc = SVG_E_DEVICE; svg_set_error("upload of the index to HBM failed"); }
		for (int k = 0; k < n && !rc; k++)
			if (hipSetDevice(devs[k]) != hipSuccess ||
			    hipMemcpy(h[k]->d_bstart, bstart, 4 * ((size_t)x->nb + 1), hipMemcpyHostToDevice) != hipSuccess) {
				rc = SVG_E_DEVICE;
				svg_set_error("upload of the index to HBM failed");
			}
		t_copy = now() - t0;
	}
	meta.join();
	free(bstart);
	munmap(x->map, x->map_len);
	x->map = NULL;
	if (!rc && meta_rc) {
		rc = meta_rc;
		svg_set_error("%s", meta_err);
	}
	for (int k = 1; k < n && !rc; k++)
		if ((rc = host_meta_copy(x, &h[k]->host))) svg_set_error("out of memory");
	if (rc) { drop_all(); return rc; }
	const double t1 = now();
	// each handle's device images (bucket code / key hash, ...), the handles side by side
	{
		std::vector<int> frc(n, 0);
		std::vector<std::string> ferr(n);
		std::vector<std::thread> ft;
		for (int k = 0; k < n; k++) {
			auto fin = [&, k] {
				frc[k] = svg_index_finish_device(h[k]);
				if (frc[k]) ferr[k] = svg_last_error();
			};
			if (n == 1) fin();
			else ft.emplace_back(fin);
		}
		for (auto &t : ft) t.join();
		for (int k = 0; k < n && !rc; k++)
			if (frc[k]) { rc = frc[k]; svg_set_error("%s", ferr[k].c_str()); }
	}
	if (rc) { drop_all(); return rc; }
	if (dbg)
		fprintf(stderr, "[svg] index block %d: %.2f GB .tab, %d handle(s), bucket walk %.3f s, keys/values in HBM %.3f s, .array + "
		        "contigs %.3f s, device images %.3f s\n", block, (double)x->map_len / 1e9, n, t_walk, t_copy, t1 - t0, now() - t1);
	for (int k = 0; k < n; k++) outs[k] = h[k];
	return 0;
}

// every block of the index, one replica per listed device (svg_index_open: one device)
static int index_open_multi(const char *prefix, const int *devs, int n, svg_index **outs)
{
	int ndev = 0;
	if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) { svg_set_error("no HIP device visible"); return SVG_E_DEVICE; }
	for (int k = 0; k < n; k++)
		if (devs[k] < 0 || devs[k] >= ndev) { svg_set_error("device %d out of range (%d visible)", devs[k], ndev); return SVG_E_ARG; }
	HIPCHK(hipSetDevice(devs[0]));
	const int nb = svg_index_count_blocks(prefix);
	if (nb < 1) { svg_set_error("index table '%s.00.b.tab' not found", prefix); return SVG_E_IO; }
	if (nb > SVG_MAX_BLOCKS) { svg_set_error("%d index blocks (at most %d)", nb, SVG_MAX_BLOCKS); return SVG_E_UNSUPPORTED; }
	int rc = index_open_block_multi(prefix, 0, devs, n, outs);
	if (rc) return rc;
	// every block stays resident in HBM (a human index is ~18 GB in all); the vote runs them in order
	std::vector<svg_index *> bk(n, (svg_index *)NULL);
	for (int b = 1; b < nb && !rc; b++) {
		if ((rc = index_open_block_multi(prefix, b, devs, n, bk.data()))) break;
		for (int k = 0; k < n; k++) {
			outs[k]->blk[b] = bk[k];
			bk[k]->stored = 1;
			outs[k]->device_bytes += bk[k]->device_bytes;
			outs[k]->nblocks = b + 1;
		}
	}
	if (rc) {
		for (int k = 0; k < n; k++) { svg_index_close(outs[k]); outs[k] = NULL; }
		return rc;
	}
	for (int k = 0; k < n; k++) outs[k]->nblocks = nb;
	return 0;
}

extern "C" int svg_index_open(const char *prefix, int device, svg_index **out)
{
	if (!prefix || !out) { svg_set_error("svg_index_open: NULL argument"); return SVG_E_ARG; }
	*out = NULL;
	return index_open_multi(prefix, &device, 1, out);
}

extern "C" int svg_index_open_devices(const char *prefix, const int *devices, int n, svg_index **out)
{
	if (!prefix || !devices || !out || n < 1 || n > 64) { svg_set_error("svg_index_open_devices: bad argument"); return SVG_E_ARG; }
	for (int k = 0; k < n; k++) out[k] = NULL;
	return index_open_multi(prefix, devices, n, out);
}

extern "C" int svg_index_export(const svg_index *h, uint32_t *bstart, int16_t *keys, uint32_t *vals, uint8_t *values,
                                uint32_t *chr_end)
{
	if (!h) { svg_set_error("svg_index_export: NULL handle"); return SVG_E_ARG; }
	HIPCHK(hipSetDevice(h->device));
	if (bstart) HIPCHK(hipMemcpy(bstart, h->d_bstart, 4 * ((size_t)h->host.nb + 1), hipMemcpyDeviceToHost));
	if (keys) HIPCHK(hipMemcpy(keys, h->d_keys, 2 * h->host.items, hipMemcpyDeviceToHost));
	if (vals) HIPCHK(hipMemcpy(vals, h->d_vals, 4 * h->host.items, hipMemcpyDeviceToHost));
	if (values) memcpy(values, h->host.values, h->host.values_bytes);
	if (chr_end) memcpy(chr_end, h->host.chr_end, 4 * (size_t)h->host.n_chr);
	return 0;
}

extern "C" void svg_index_close(svg_index *h)
{
	if (!h) return;
	for (int k = 1; k < h->nblocks && k < SVG_MAX_BLOCKS; k++) svg_index_close(h->blk[k]);
	hipSetDevice(h->device);
	if (h->stream) hipStreamSynchronize(h->stream);
	if (h->stream2) hipStreamSynchronize(h->stream2);
	if (h->up_stream) hipStreamSynchronize(h->up_stream);
	if (h->down_stream) hipStreamSynchronize(h->down_stream);
	svg_io_free(h);
	svg_long_ws_free(h);
	for (int s = 0; s < 3; s++) {
		hipFree(h->d_prec[s]);
		hipFree(h->d_lane[s]);
		hipFree(h->d_big[s]);
		hipFree(h->d_in[s]);
		hipFree(h->d_out[s]);
		hipEvent_t *evs[6] = {h->ev_lane, h->ev_wave, h->ev_probe, h->ev_up, h->ev_done, h->ev_down};
		for (int k = 0; k < 6; k++)
			if (evs[k][s]) hipEventDestroy(evs[k][s]);
	}
	hipFree(h->d_lscratch);
	for (int k = 0; k < 4; k++)
		for (int i = 0; i < 64; i++)
			for (int j = 0; j < 2; j++)
				if (h->tev[k][i][j]) hipEventDestroy(h->tev[k][i][j]);
	hipFree(h->d_bstart); hipFree(h->d_keys); hipFree(h->d_vals); hipFree(h->d_values); hipFree(h->d_chr);
	hipFree(h->d_bgrp); hipFree(h->d_keys8); hipFree(h->d_bline); hipFree(h->d_bcode); hipFree(h->d_khash); hipFree(h->d_ksorted);
	hipFree(h->d_scratch); hipFree(h->d_stats); hipFree(h->d_err);
	if (h->ev_last) hipEventDestroy(h->ev_last);
	streams_release(h);
	svg_host_index_free(&h->host);
	free(h);
}

extern "C" int svg_index_get_info(const svg_index *h, svg_index_info *o)
{
	if (!h || !o) { svg_set_error("svg_index_get_info: NULL argument"); return SVG_E_ARG; }
	o->items = h->host.items;
	o->buckets = h->host.nb;
	o->index_gap = h->host.gap;
	o->padding = h->host.padding;
	o->array_length = h->host.length;
	o->n_chromosomes = h->host.n_chr;
	o->device_bytes = h->device_bytes;
	o->device = h->device;
	o->array_values_bytes = h->host.values_bytes;
	o->n_blocks = h->nblocks > 1 ? h->nblocks : 1;
	return 0;
}

// ------------------------------------------------------------------ per-kernel timing
static int timing_fold(svg_index *h, int k)
{
	for (int i = 0; i < h->tn[k]; i++) {
		float ms = 0.f;
		HIPCHK(hipEventSynchronize(h->tev[k][i][1]));
		HIPCHK(hipEventElapsedTime(&ms, h->tev[k][i][0], h->tev[k][i][1]));
		h->tms[k] += ms;
	}
	h->tn[k] = 0;
	return 0;
}

// bracket one launch of kind k (0 probe, 1 vote, 2 gather, 3 lane): phase 0 before, 1 after
static int timing_mark(svg_index *h, int k, int phase, hipStream_t st)
{
	if (!h->timing) return 0;
	if (phase == 0 && h->tn[k] == 64) { int rc = timing_fold(h, k); if (rc) return rc; }
	HIPCHK(hipEventRecord(h->tev[k][h->tn[k]][phase], st));
	if (phase == 1) { h->tn[k]++; h->tcount[k]++; }
	return 0;
}

extern "C" int svg_set_timing(svg_index *h, int enable)
{
	if (!h) { svg_set_error("svg_set_timing: NULL handle"); return SVG_E_ARG; }
	HIPCHK(hipSetDevice(h->device));
	if (enable && !h->timing) {
		for (int k = 0; k < 4; k++)
			for (int i = 0; i < 64; i++)
				for (int j = 0; j < 2; j++)
					if (!h->tev[k][i][j]) HIPCHK(hipEventCreate(&h->tev[k][i][j]));
	}
	h->timing = enable ? 1 : 0;
	for (int k = 0; k < 4; k++) { h->tn[k] = 0; h->tcount[k] = 0; h->tms[k] = 0.0; }
	for (int k = 1; k < h->nblocks; k++) {
		int rc = svg_set_timing(h->blk[k], enable);
		if (rc) return rc;
	}
	return 0;
}

// fold every block's pending events; per-kind totals over the blocks
static int timing_total(svg_index *h, double ms[4], int launches[4])
{
	for (int k = 0; k < 4; k++) { ms[k] = 0.0; launches[k] = 0; }
	for (int b = 0; b < h->nblocks; b++) {
		svg_index *x = b ? h->blk[b] : h;
		for (int k = 0; k < 4; k++) {
			int rc = timing_fold(x, k);
			if (rc) return rc;
			ms[k] += x->tms[k];
			launches[k] += x->tcount[k];
		}
	}
	return 0;
}

int svg_timing_mark(svg_index *h, int k, int phase, hipStream_t st) { return timing_mark(h, k, phase, st); }

extern "C" int svg_get_timing(svg_index *h, double *probe_ms, double *vote_ms, int *probe_launches, int *vote_launches)
{
	if (!h) { svg_set_error("svg_get_timing: NULL handle"); return SVG_E_ARG; }
	HIPCHK(hipSetDevice(h->device));
	double ms[4];
	int n[4];
	int rc = timing_total(h, ms, n);
	if (rc) return rc;
	// vote = everything after the probe kernel (gather, lane and the wave kernel)
	if (probe_ms) *probe_ms = ms[0];
	if (vote_ms) *vote_ms = ms[1] + ms[2] + ms[3];
	if (probe_launches) *probe_launches = n[0];
	if (vote_launches) *vote_launches = n[1];
	return 0;
}

extern "C" int svg_get_kernel_timing(svg_index *h, double ms[4], int launches[4])
{
	if (!h || !ms || !launches) { svg_set_error("svg_get_kernel_timing: NULL argument"); return SVG_E_ARG; }
	HIPCHK(hipSetDevice(h->device));
	return timing_total(h, ms, launches);
}

extern "C" int svg_set_stats(svg_index *h, int enable)
{
	if (!h) return SVG_E_ARG;
	h->stats_on = enable ? 1 : 0;
	return 0;
}

// debug: raw device counters (32 words; 8..15 = per-phase wave cycles in SVG_STAMPS builds,
// 16..20 = light lane pass: deferrals by reason (candidates > CAP or length, slots > K,
// shift-indel), candidates voted, deferrals; 21..25 = the same for the heavy lane pass;
// 26 / 27 = wave-kernel candidates settled by batch mode / replayed serially)
extern "C" int svg_debug_counters(svg_index *h, unsigned long long *out32)
{
	if (!h || !out32) return SVG_E_ARG;
	HIPCHK(hipMemcpy(out32, h->d_stats, 32 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
	return 0;
}

// waits for the handle's queued work and reports (and clears) the sticky device error word
extern "C" int svg_device_status(svg_index *h)
{
	if (!h) { svg_set_error("svg_device_status: NULL handle"); return SVG_E_ARG; }
	HIPCHK(hipSetDevice(h->device));
	if (h->last_pending) HIPCHK(hipEventSynchronize(h->ev_last));
	uint32_t e = 0;
	for (int k = 0; k < h->nblocks; k++) {
		svg_index *b = k ? h->blk[k] : h;
		if (k && b->last_pending) HIPCHK(hipEventSynchronize(b->ev_last));
		uint32_t eb = 0;
		HIPCHK(hipMemcpy(&eb, b->d_err, 4, hipMemcpyDeviceToHost));
		if (eb) HIPCHK(hipMemset(b->d_err, 0, 4));
		e |= eb;
	}
	if (!e) return 0;
	if (e & 1u) svg_set_error("a read needs more subread probes than the read-length bound of svg_set_max_read_length "
	                          "(%d) provides; its records were zeroed", h->max_read_len);
	else svg_set_error("a read is longer than the kernel variant's text buffer; its records were zeroed");
	return SVG_E_ARG;
}

extern "C" int svg_get_stats(const svg_index *h, svg_batch_stats *o)
{
	if (!h || !o) return SVG_E_ARG;
	*o = h->last_stats;
	return 0;
}

// largest applied_subreads * gap over read lengths 15+gap..max_len (core.c:3117-3129)
static int svg_probe_bound(int max_len, int gap, int n)
{
	int best = 0;
	for (int len = 15 + gap; len <= max_len; len++) {
		int cr = (len - 15 - gap) << 16, step;
		if (len <= 160) { step = cr / (n - 1); if (step < (gap << 16)) step = gap << 16; }
		else { step = 6 << 16; if (cr / step > 62) step = cr / 62; }
		int np = (1 + cr / step) * gap;
		if (np > best) best = np;
	}
	return best;
}

extern "C" int svg_set_max_read_length(svg_index *h, int max_len)
{
	if (!h || max_len < 1 || max_len > SVG_MAX_READ_LENGTH) { svg_set_error("svg_set_max_read_length: bad argument"); return SVG_E_ARG; }
	h->max_read_len = max_len;
	return 0;
}

int svg_check_params(const svg_index *h, const svg_params *p, int paired)
{
	if (p->multi_best < 1 || p->multi_best > 3) { svg_set_error("multi_best must be 1..3"); return SVG_E_UNSUPPORTED; }
	if (p->top_scores != 3) { svg_set_error("top_scores must be 3 (reference runtime value)"); return SVG_E_UNSUPPORTED; }
	if (p->max_vote_combinations < 1 || p->max_vote_combinations > 3) { svg_set_error("max_vote_combinations must be 1..3"); return SVG_E_UNSUPPORTED; }
	if (p->max_vote_simples < 1 || p->max_vote_simples > 64) { svg_set_error("max_vote_simples must be 1..64"); return SVG_E_UNSUPPORTED; }
	if (p->max_vote_simples > 16 && !paired) { svg_set_error("single-end max_vote_simples must be <= 16"); return SVG_E_UNSUPPORTED; }
	if (p->total_subreads < 2 || p->total_subreads > 64) { svg_set_error("total_subreads must be 2..64"); return SVG_E_UNSUPPORTED; }
	if (p->max_indel_length < 0) { svg_set_error("max_indel_length < 0"); return SVG_E_ARG; }
	if (p->do_big_margin_filtering_for_junctions && (p->big_margin_record_size < 0 || p->big_margin_record_size > SVG_BIG_MARGIN_WORDS ||
	                                                 (p->big_margin_record_size >= 3 && p->big_margin_record_size % 3))) {
		svg_set_error("big_margin_record_size must be 0, 1, 2, 3, 6 or 9"); return SVG_E_UNSUPPORTED;
	}
	if (p->do_breakpoint_detection && p->max_insertion_at_junctions != 0) {
		svg_set_error("max_insertion_at_junctions > 0 reads past the read end in the reference; not supported"); return SVG_E_UNSUPPORTED;
	}
	(void)h;
	return 0;
}

template <int ENDS, int MAXL, int MAXP, int WPB, int OCC, bool SJ>
static int launch_t(svg_index *h, KParams &kp, hipStream_t st)
{
	typedef WaveLDS<ENDS, MAXL, MAXP, SJ> LT;
	size_t lds = (size_t)WPB * ((sizeof(LT) + 15) & ~(size_t)15);
	int per_cu = (int)(160 * 1024 / lds);
	if (per_cu < 1) { svg_set_error("kernel LDS too large"); return SVG_E_DEVICE; }
	if (per_cu > 4 * OCC / WPB) per_cu = 4 * OCC / WPB;   // 4 SIMDs x OCC waves
	if (h->wave_cap > 0 && per_cu > h->wave_cap) per_cu = h->wave_cap;
	if (svg_get_option("debug") & 1)
		fprintf(stderr, "[svg] vote_kernel<%d,%d,%d,%d,%d,%d>: LDS %zu B/wave, %d blocks/CU\n", ENDS, MAXL,
		        MAXP, WPB, OCC, (int)SJ, sizeof(LT), per_cu);
	uint64_t blocks = (uint64_t)h->n_cu * per_cu;
	uint64_t need = (kp.n_reads + WPB - 1) / WPB;
	if (blocks > need) blocks = need;
	if (blocks < 1) blocks = 1;
	size_t per_end = (size_t)NSLOT * COLD_WORDS + NSLOT;
	size_t words = blocks * WPB * (ENDS * per_end + (ENDS == 2 ? (size_t)NSLOT * 4 : 0));
	if (words > h->scratch_words) {
		hipFree(h->d_scratch);
		h->d_scratch = NULL;
		h->scratch_words = 0;
		if (dmalloc(h, (void **)&h->d_scratch, words * 4 + 65536)) return SVG_E_NOMEM;
		h->scratch_words = words;
	}
	kp.scratch = h->d_scratch;
	hipLaunchKernelGGL((vote_kernel<ENDS, MAXL, MAXP, WPB, OCC, SJ>), dim3((unsigned)blocks), dim3(64 * WPB), lds, st, kp);
	HIPCHK(hipGetLastError());
	return 0;
}


// kernel variant by mode and announced read-length bound
static int launch_vote(svg_index *h, KParams &kp, hipStream_t st, int npmax, bool sj, int ends)
{
	// subjunc (junction minor search, donor scoring, big-margin records) is a separate
	// variant so the plain-align kernels carry none of its registers
	if (sj) {
		if (h->max_read_len > 256 || npmax > 64) {
			// long reads (161..1209 bp): text of both strands in LDS for donor scoring
			if (ends == 2) return npmax <= 64 ? launch_t<2, 1216, 64, 2, 4, true>(h, kp, st) : launch_t<2, 1216, 192, 2, 4, true>(h, kp, st);
			return npmax <= 64 ? launch_t<1, 1216, 64, 2, 4, true>(h, kp, st) : launch_t<1, 1216, 192, 2, 4, true>(h, kp, st);
		}
#ifndef SVG_PESJ_OCC
#define SVG_PESJ_OCC 4
#endif
		if (ends == 2)
			return npmax <= 32 ? launch_t<2, 256, 32, 2, SVG_PESJ_OCC, true>(h, kp, st) : launch_t<2, 256, 64, 2, SVG_PESJ_OCC, true>(h, kp, st);
		return npmax <= 32 ? launch_t<1, 256, 32, 2, 4, true>(h, kp, st) : launch_t<1, 256, 64, 2, 4, true>(h, kp, st);
	}
	if (h->max_read_len > 256 || npmax > 64) {
		// long reads (161..1210 bp: 6 bp subread step, <= 63 subreads per gap slot)
		if (ends == 2) return npmax <= 64 ? launch_t<2, 1216, 64, 2, 4, false>(h, kp, st) : launch_t<2, 1216, 192, 2, 4, false>(h, kp, st);
		return npmax <= 64 ? launch_t<1, 1216, 64, 2, 4, false>(h, kp, st) : launch_t<1, 1216, 192, 2, 4, false>(h, kp, st);
	}
	if (ends == 2) return npmax <= 32 ? launch_t<2, 256, 32, 1, 4, false>(h, kp, st) : launch_t<2, 256, 64, 1, 4, false>(h, kp, st);
#ifndef SVG_WAVE_CAP
#define SVG_WAVE_CAP 6   // C3: 317 (uncapped, 10) -> 328 Mreads/s; 4 and 3 starve the wave kernel
#endif
#ifndef SVG_SE_OCC
#define SVG_SE_OCC 7   // 72 VGPRs: the wave kernel shares the CUs with the next chunk's probe / lane kernels (round 3, C3: OCC 4 139, 5 116, 6 108, 8 134 ms/step; round 6 after the batch-mode table: 6 92.3, 7 89.0)
#endif
	return npmax <= 32 ? launch_t<1, 256, 32, 2, SVG_SE_OCC, false>(h, kp, st) : launch_t<1, 256, 64, 2, SVG_SE_OCC, false>(h, kp, st);
}

// ------------------------------------------------------------------ batch set-up and chunk launch
// svg_vote_prepare checks a batch and fills the kernel parameters; svg_vote_chunk launches the
// probe and lane kernels of reads [c0, c0+cn) on st (records in slot `slot`) and the wave
// kernel on st2 (event handoff when st2 != st).  svg_vote_batch_device drives the chunks of one
// call; the host-buffer pipeline (svg_io.hip) drives one chunk per sub-batch with its own slots.
int svg_vote_prepare(svg_index *h, const svg_params *p, const svg_reads *r1, const svg_reads *r2, svg_mapping_result *out,
                     svg_subjunc_result *jout, uint16_t *big_margin, VoteJob *job)
{
	if (!h || !p || !r1 || !out) { svg_set_error("svg_vote_batch_device: NULL argument"); return SVG_E_ARG; }
	if (r2 && r2->n_reads != r1->n_reads) { svg_set_error("R1/R2 read counts differ"); return SVG_E_ARG; }
	int rc = svg_check_params(h, p, r2 != NULL);
	if (rc) return rc;
	if (p->do_breakpoint_detection && !jout) { svg_set_error("do_breakpoint_detection needs jout"); return SVG_E_ARG; }
	if (p->do_big_margin_filtering_for_junctions && !big_margin) { svg_set_error("big-margin filtering needs big_margin"); return SVG_E_ARG; }
	// subjunc reads > 160 bp: the reference also runs fragile junction voting (gehash_go_q,
	// core_fragile_junction_voting, core-junction.c:5151-5424) on them, which only adds junction
	// and indel events to the event tables (host post-processing, outside this boundary); the
	// vote records come from the regular voting below (long-read junction branch included)
	KParams &kp = job->kp;
	memset(&kp, 0, sizeof kp);
	kp.err = h->d_err;
	kp.p = *p;
	kp.ix = h->dix;
	// one-hit records carry positions only when the line kernel probes the inline key-hash image
	kp.seq1 = r1->seq; kp.off1 = r1->offsets; kp.len1 = r1->lens;
	if (r2) { kp.seq2 = r2->seq; kp.off2 = r2->offsets; kp.len2 = r2->lens; }
	kp.n_reads = r1->n_reads;
	kp.out = (uint8_t *)out;
	kp.jout = (uint8_t *)jout;
	kp.bm_out = big_margin;
	kp.tol = p->max_indel_length < 16 ? p->max_indel_length : 16;
	kp.ii_end = 5;
	if (kp.tol > 5) kp.ii_end = (kp.tol % 5) ? (kp.tol - kp.tol % 5 + 5) : kp.tol;
	kp.low = h->dix.start_base_offset;
	kp.high = h->dix.start_base_offset + h->dix.length;
	kp.stats = h->stats_on ? h->d_stats : NULL;
	// probes per strand are bounded by the read lengths the caller announced
	job->npmax = svg_probe_bound(h->max_read_len, h->dix.gap, p->total_subreads);
	job->sj = p->do_breakpoint_detection || p->do_big_margin_filtering_for_junctions;
	if (job->npmax > 192) { svg_set_error("%d subreads per strand exceed 192", job->npmax); return SVG_E_UNSUPPORTED; }
	job->ends = r2 ? 2 : 1;
	// phase P as its own kernel per chunk of reads (<= 1 GiB of probe records), then the vote
	// kernels on its records
	const int nps = job->npmax > 0 ? job->npmax : 1;
	job->nps = nps;
	job->per_read = (uint64_t)job->ends * 2 * nps;
	uint64_t chunk = ((uint64_t)1 << 30) / (job->per_read * 8);
	if (chunk > (uint64_t)0x7fffffff / job->per_read) chunk = (uint64_t)0x7fffffff / job->per_read;
	{ const int64_t oc = svg_get_option("chunk"); if (oc > 0 && (uint64_t)oc < chunk) chunk = (uint64_t)oc; }   // testing
	if (chunk < 1) chunk = 1;
	job->chunk = chunk;
	// chunk pipeline: the wave kernel of chunk c runs on stream2 while the probe and lane kernels
	// of chunk c+1 run on st; slot c & 1 holds a chunk's probe records and lane buffers until its
	// wave kernel is done.  On by default for single-end align only (C3: 289 -> 304 Mreads/s; PE
	// and subjunc, whose wave kernels are 2-3x longer, lost 1-2%: the kernels time-share the CUs
	// there).  Option "overlap" 0/1 forces it off/on.
	const int64_t oo = svg_get_option("overlap");
	job->overlap_mode = oo >= 0 ? oo == 1 : (!job->sj && !r2);
	PParams &pp = job->pp;
	memset(&pp, 0, sizeof pp);
	pp.ix = h->dix;
	pp.seq1 = kp.seq1; pp.seq2 = kp.seq2;
	pp.nps = nps;
	pp.total_subreads = p->total_subreads; pp.reverse_r1 = p->reverse_r1; pp.reverse_r2 = p->reverse_r2;
	pp.nb_magic = ~0ull / h->dix.nb + 1;   // ceil(2^64 / nb), nb is not a power of two
	pp.stats = kp.stats;
	// align mode, reads <= 160 bp: lane-per-read (SE) / lane-per-pair (PE) fast path
	// (svg_lane.hip), probe records in SoA layout
	job->lane = svg_lane_eligible(h, p, r2 != NULL, job->sj) != 0 && (!r2 || nps <= (job->sj ? 14 : 10)) && (!job->sj || nps <= 14) &&
	            !h->stored;   // later blocks of a multi-block index merge with stored records: wave kernel
	kp.stored = h->stored;
	pp.soa = job->lane ? 1 : 0;
	pp.window = h->dix.nb >= 131073u;   // key_hi <= 32767: int16 order == key order
	pp.readmajor = 1;
	return 0;
}

// reads [c0, c0+cn) of the prepared batch; slot's probe records / lane buffers must be free
int svg_vote_chunk(svg_index *h, VoteJob *job, uint64_t c0, uint64_t cn, int slot, hipStream_t st, hipStream_t st2)
{
	int rc = svg_vote_chunk_probe(h, job, c0, cn, slot, st);
	return rc ? rc : svg_vote_chunk_vote(h, job, c0, cn, slot, st, st2);
}

int svg_vote_chunk_probe(svg_index *h, VoteJob *job, uint64_t c0, uint64_t cn, int slot, hipStream_t st)
{
	if (slot < 0 || slot > 2) { svg_set_error("chunk slot %d out of range", slot); return SVG_E_ARG; }   // [3]-slot buffers
	const KParams &kp = job->kp;
	int rc;
	if ((rc = svg_ensure(h, &h->d_prec[slot], &h->prec_cap[slot], cn * job->per_read * 8))) return rc;
	PParams pp = job->pp;
	pp.out = (uint2 *)h->d_prec[slot];
	pp.off1 = kp.off1 + c0; pp.len1 = kp.len1 + c0;
	if (kp.len2) { pp.off2 = kp.off2 + c0; pp.len2 = kp.len2 + c0; }
	pp.n_reads = (uint32_t)cn;
	uint64_t pb = (cn * job->per_read + 255) / 256, pmax = (uint64_t)h->n_cu * 32;
	if (pb > pmax) pb = pmax;
	if ((rc = timing_mark(h, 0, 0, st))) return rc;
	// 8 blocks of 256 per CU (<= 64 VGPRs): the probe chain is latency-bound, occupancy is what
	// hides it (C3: 11.3 ms at 4 waves/SIMD, 8.7 ms at 8); bucket-line image (one random 64-B
	// line per probe) when the index has one
	const bool pe = kp.len2 != NULL;
	if (pp.packed) {
		// 2-bit input: chunk-relative read starts
		for (int e = 0; e < (pe ? 2 : 1); e++) {
			if (pp.pk_starts[e]) pp.pk_starts[e] += c0;
			else pp.pk_base0[e] += c0 * pp.pk_stride[e];
		}
	}
#define PROBE_LAUNCH(E, L, P) hipLaunchKernelGGL((probe_kernel<E, 8, L, P>), dim3((unsigned)pb), dim3(256), 0, st, pp)
	if (h->dix.bline || h->dix.bcode || h->dix.khash) {
		// bucket lines: grouped probe kernel + the big-bucket kernel on its list
		pp.group = (uint32_t)(PROBE_GROUP_RECS / job->per_read);
		if (pp.group > 64) pp.group = 64;
		if (pp.group < 1) pp.group = 1;
		const uint64_t ng = (cn + pp.group - 1) / pp.group;
		// grid: 32 blocks per CU (4 rounds of the 8 resident); option probe_cap sets blocks per CU
		const int64_t pc = svg_get_option("probe_cap");
		uint64_t gb = ng, gmax = (uint64_t)h->n_cu * (pc > 0 ? (uint64_t)pc : 32u);
		if (gb > gmax) gb = gmax;
		// one list region per line-kernel block, sized for all of its probes; per-block counts
		const uint64_t per_blk = (ng + gb - 1) / gb, stride = per_blk * pp.group * job->per_read;
		const uint64_t cnt_words = (gb + 63) & ~63ull;
		if ((rc = svg_ensure(h, &h->d_big[slot], &h->big_cap[slot], (cnt_words + gb * stride) * 4 + 256))) return rc;
		pp.big_count = (uint32_t *)h->d_big[slot];
		pp.big_list = (uint32_t *)h->d_big[slot] + cnt_words;
		pp.big_stride = (uint32_t)stride;
		pp.big_regions = (uint32_t)gb;
#define LINE_LAUNCH(E, P, C) hipLaunchKernelGGL((probe_line_kernel<E, P, C>), dim3((unsigned)gb), dim3(256), 0, st, pp)
		if (h->dix.khash) {
			if (pp.packed) { if (pe) LINE_LAUNCH(2, true, IMG_KHASH); else LINE_LAUNCH(1, true, IMG_KHASH); }
			else { if (pe) LINE_LAUNCH(2, false, IMG_KHASH); else LINE_LAUNCH(1, false, IMG_KHASH); }
		} else if (h->dix.bcode) {
			if (pp.packed) { if (pe) LINE_LAUNCH(2, true, IMG_CODE); else LINE_LAUNCH(1, true, IMG_CODE); }
			else { if (pe) LINE_LAUNCH(2, false, IMG_CODE); else LINE_LAUNCH(1, false, IMG_CODE); }
		} else {
			if (pp.packed) { if (pe) LINE_LAUNCH(2, true, IMG_LINE); else LINE_LAUNCH(1, true, IMG_LINE); }
			else { if (pe) LINE_LAUNCH(2, false, IMG_LINE); else LINE_LAUNCH(1, false, IMG_LINE); }
		}
#undef LINE_LAUNCH
		HIPCHK(hipGetLastError());
		// (the key-hash image resolves every probe in the line kernel: no big-bucket list)
		if (!h->dix.khash) hipLaunchKernelGGL(probe_big_kernel, dim3((unsigned)(h->n_cu * 8)), dim3(256), 0, st, pp);
	} else if (h->dix.bline) {
		if (pp.packed) { if (pe) PROBE_LAUNCH(2, true, true); else PROBE_LAUNCH(1, true, true); }
		else { if (pe) PROBE_LAUNCH(2, true, false); else PROBE_LAUNCH(1, true, false); }
	} else {
		if (pp.packed) { if (pe) PROBE_LAUNCH(2, false, true); else PROBE_LAUNCH(1, false, true); }
		else { if (pe) PROBE_LAUNCH(2, false, false); else PROBE_LAUNCH(1, false, false); }
	}
#undef PROBE_LAUNCH
	HIPCHK(hipGetLastError());
	return timing_mark(h, 0, 1, st);
}

int svg_vote_chunk_vote(svg_index *h, VoteJob *job, uint64_t c0, uint64_t cn, int slot, hipStream_t st, hipStream_t st2)
{
	const KParams &kp = job->kp;
	const svg_params *p = &kp.p;
	const int ends = job->ends, nps = job->nps;
	const bool pe = kp.len2 != NULL;
	int rc;
	// overlapped, the wave kernel leaves CU slots to the next chunk's probe kernel, whose
	// latency-bound chain needs the occupancy (the wave kernel has slack on its stream)
	h->wave_cap = 0;
	if (st2 != st) {
		const int64_t ow = svg_get_option("wave_cap");
		h->wave_cap = ow >= 0 ? (int)ow : SVG_WAVE_CAP;
	}
	KParams kc = kp;
	kc.off1 = kp.off1 + c0; kc.len1 = kp.len1 + c0;
	if (pe) { kc.off2 = kp.off2 + c0; kc.len2 = kp.len2 + c0; }
	kc.n_reads = cn;
	kc.out = kp.out + c0 * ends * p->multi_best * 68;
	if (kp.jout) kc.jout = kp.jout + c0 * ends * p->multi_best * 16;
	if (kp.bm_out) kc.bm_out = kp.bm_out + c0 * ends * SVG_BIG_MARGIN_WORDS;
	kc.precs = (const uint2 *)h->d_prec[slot];
	kc.nps = nps;
	if (job->lane) {
		// gather + lane kernels vote every read they can; the rest (deferral list) go to
		// vote_kernel below, which reads the SoA probe records of the deferred reads
		uint32_t *dl = NULL, *dc = NULL;
		rc = pe ? svg_lane_pe_chunk(h, slot, p, kc.len1, kc.len2, (uint32_t)cn, kc.precs, nps, kc.out, job->sj ? kc.jout : NULL,
		                            kc.bm_out, kc.seq1, kc.off1, kc.seq2, kc.off2, kp.stats, &dl, &dc, st)
		        : svg_lane_chunk(h, slot, p, kc.len1, (uint32_t)cn, kc.precs, nps, kc.out, job->sj ? kc.jout : NULL, kc.bm_out,
		                         kc.seq1, kc.off1, kp.stats, &dl, &dc, st);
		if (rc) return rc;
		kc.prec_stride = (uint32_t)cn;
		kc.idx = dl;
		kc.idx_count = dc;
		kc.work = dc + 2;
		{   // option wave_static: eighths of the deferral list dealt out without the work counter.
			// Single-end: 6 (C3 1.67 -> 1.535 ms per wave-kernel launch); pairs, whose deferred
			// reads cost far more and vary more: 0, all from the counter (C4 with 6: 272 vs 235
			// ms/step, profiles/r04/r/bench_c4.json)
			const int64_t ws = svg_get_option("wave_static");
			kc.static_eighths = ws >= 0 && ws <= 8 ? (int32_t)ws : (ends == 1 ? 6 : 0);
		}
	}
	if (st2 != st) {
		HIPCHK(hipEventRecord(h->ev_lane[slot], st));
		HIPCHK(hipStreamWaitEvent(st2, h->ev_lane[slot], 0));
	}
	if ((rc = timing_mark(h, 1, 0, st2))) return rc;
	rc = launch_vote(h, kc, st2, job->npmax, job->sj, ends);
	if (!rc) rc = timing_mark(h, 1, 1, st2);
	return rc;
}

static int vote_batch_device(svg_index *h, const svg_params *p, const svg_reads *r1, const svg_reads *r2,
                             const svg_packed_reads *pk, svg_mapping_result *out, svg_subjunc_result *jout,
                             uint16_t *big_margin, void *stream)
{
	VoteJob job;
	int rc = svg_vote_prepare(h, p, r1, r2, out, jout, big_margin, &job);
	if (rc) return rc;
	if (pk) {
		job.pp.packed = 1;
		for (int e = 0; e < (r2 ? 2 : 1); e++) {
			job.pp.pk_bases[e] = pk[e].bases;
			job.pp.pk_xmask[e] = pk[e].xmask;
			job.pp.pk_starts[e] = pk[e].starts;
			job.pp.pk_stride[e] = pk[e].stride;
			job.pp.pk_base0[e] = 0;
		}
	}
	HIPCHK(hipSetDevice(h->device));
	hipStream_t st = stream ? (hipStream_t)stream : h->stream;
	if (r1->n_reads == 0) return 0;
	// the handle's buffers (probe records, lane lists, scratch) are shared by every call: this
	// call's work starts after the previous call's, whatever streams the two were given
	if (h->last_pending) HIPCHK(hipStreamWaitEvent(st, h->ev_last, 0));
	if (h->stats_on) HIPCHK(hipMemsetAsync(h->d_stats, 0, 32 * sizeof(unsigned long long), st));
	// chunks of <= 160 MiB of probe records (1M single-end 100-bp reads, the host pipeline's
	// sub-batch): the records stay in the 256 MB infinity cache between the probe kernel that
	// writes them and the lane / wave kernels that read them (option "chunk" sets the chunk instead)
	uint64_t chunk = job.chunk;
	if (svg_get_option("chunk") <= 0) {
		const uint64_t cc = ((uint64_t)160 << 20) / (job.per_read * 8);
		if (cc >= 1 && cc < chunk) chunk = cc;
	}
	const uint64_t n = r1->n_reads;
	const bool overlap = job.overlap_mode && chunk < n;
	hipStream_t st2 = overlap ? h->stream2 : st;
	if (svg_get_option("debug") & 1)
		fprintf(stderr, "[svg] batch of %llu reads: chunks of %llu, chunk pipeline %s\n", (unsigned long long)n,
		        (unsigned long long)chunk, overlap ? "on" : "off");
	// chunk slots (probe records, lane lists): 2, as in the host pipeline (three were measured slower
	// there -- the records must stay in the infinity cache)
	const int NS = 2;
	bool slot_busy[3] = {false, false, false};
	// chunk boundaries: ramped at both ends (chunk/4, chunk/2 first and last, option host_ramp) when
	// the batch holds at least 8 chunks -- the second stream gets work sooner and the last wave
	// kernel, which nothing overlaps, is short
	std::vector<uint64_t> cb{0};
	{
		const bool ramp = overlap && svg_get_option("host_ramp") != 0 && n >= 8 * chunk && chunk >= 64;
		const uint64_t q4 = chunk / 4, q2 = chunk / 2;
		if (ramp) { cb.push_back(q4); cb.push_back(q4 + q2); }
		const uint64_t body_end = n - (ramp ? q2 + q4 : 0);
		while (cb.back() < body_end) cb.push_back(cb.back() + chunk < body_end ? cb.back() + chunk : body_end);
		if (ramp) { cb.push_back(body_end + q2); cb.push_back(n); }
	}
	// option dev_pace: the host thread enqueues chunk k only once chunk k-2's wave kernel is done, as
	// the host pipeline's thread does (it waits on sub-batch i-2 before it queues i): fewer kernels
	// of later chunks queued behind the running ones
	const bool pace = overlap && svg_get_option("dev_pace") > 0;
	for (size_t k = 0; k + 1 < cb.size() && !rc; k++) {
		const uint64_t c0 = cb[k], cn = cb[k + 1] - cb[k];
		const int slot = overlap ? (int)(k % (size_t)NS) : 0;
		if (pace && slot_busy[slot]) HIPCHK(hipEventSynchronize(h->ev_wave[slot]));
		if (slot_busy[slot]) HIPCHK(hipStreamWaitEvent(st, h->ev_wave[slot], 0));
		rc = svg_vote_chunk(h, &job, c0, cn, slot, st, st2);
		if (!rc && overlap) {
			HIPCHK(hipEventRecord(h->ev_wave[slot], st2));
			slot_busy[slot] = true;
		}
	}
	// join: the caller's stream sees every wave kernel of the batch
	for (int s = 0; s < NS && overlap; s++)
		if (slot_busy[s]) HIPCHK(hipStreamWaitEvent(st, h->ev_wave[s], 0));
	if (rc) return rc;
	HIPCHK(hipEventRecord(h->ev_last, st));
	h->last_pending = 1;
	if (h->stats_on) {
		unsigned long long s[5];
		HIPCHK(hipMemcpyAsync(s, h->d_stats, sizeof s, hipMemcpyDeviceToHost, st));
		HIPCHK(hipStreamSynchronize(st));
		h->last_stats.probes = s[0];
		h->last_stats.bucket_items = s[1];
		h->last_stats.hits = s[2];
		h->last_stats.results = s[3];
		h->last_stats.deferred = s[4];
	}
	return 0;
}

// multi-block index: block 0 (this handle), then blocks 1.. in order on the same stream, each
// merging with the records the previous blocks left (read_chunk_circles, core.c:3567-3613)
static int vote_blocks(svg_index *h, const svg_params *p, const svg_reads *r1, const svg_reads *r2,
                       const svg_packed_reads *pk, svg_mapping_result *out, svg_subjunc_result *jout,
                       uint16_t *big_margin, void *stream)
{
	int rc = vote_batch_device(h, p, r1, r2, pk, out, jout, big_margin, stream);
	if (rc || h->nblocks < 2) return rc;
	svg_batch_stats acc = h->last_stats;
	void *st = stream ? stream : (void *)h->stream;
	for (int k = 1; k < h->nblocks && !rc; k++) {
		svg_index *b = h->blk[k];
		b->max_read_len = h->max_read_len;
		b->stats_on = h->stats_on;
		rc = vote_batch_device(b, p, r1, r2, pk, out, jout, big_margin, st);
		if (!rc && h->stats_on) {
			acc.probes += b->last_stats.probes; acc.bucket_items += b->last_stats.bucket_items;
			acc.hits += b->last_stats.hits; acc.results = b->last_stats.results;
			acc.deferred += b->last_stats.deferred;
		}
	}
	if (h->stats_on) h->last_stats = acc;
	// later calls on this handle wait for the last block's work
	if (!rc) {
		HIPCHK(hipEventRecord(h->ev_last, (hipStream_t)st));
		h->last_pending = 1;
	}
	return rc;
}

extern "C" int svg_vote_batch_device(svg_index *h, const svg_params *p, const svg_reads *r1, const svg_reads *r2,
                                     svg_mapping_result *out, svg_subjunc_result *jout, uint16_t *big_margin, void *stream)
{
	return vote_blocks(h, p, r1, r2, NULL, out, jout, big_margin, stream);
}

// align mode from 2-bit packed device reads: r1/r2 carry the lengths, pk[e] the codes
int svg_vote_batch_device_packed(svg_index *h, const svg_params *p, const svg_reads *r1, const svg_reads *r2,
                                 const svg_packed_reads *pk, svg_mapping_result *out, svg_subjunc_result *jout,
                                 uint16_t *big_margin, hipStream_t stream)
{
	return vote_blocks(h, p, r1, r2, pk, out, jout, big_margin, (void *)stream);
}
