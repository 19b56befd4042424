// svg_device.h -- HIP-side internals shared by the vote kernels and the GPU index builder.
#ifndef SVG_DEVICE_H
#define SVG_DEVICE_H
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "subread_vote.h"
#include "svg_internal.h"

// ---------------------------------------------------------------------------------------------
// device-side index
struct DevIndex {
	const uint32_t *bstart;   // nb+1
	const int16_t *keys;
	const uint32_t *vals;
	const uint8_t *values;    // .array
	const uint32_t *chr_end;  // .reads offsets
	uint32_t nb, n_chr;
	uint32_t start_point, length, start_base_offset, values_bytes;
	int32_t gap, padding;
	// compact probe images (device only; NULL when absent, i.e. nb < 16843009):
	//   bgrp[g]: 8 words per 16 buckets: first item of bucket 16g, then 16 u8 item counts
	//            (255 = 255 or more: use bstart/keys for that bucket); small enough to stay
	//            in the Infinity Cache
	//   keys8[i] = keys[i] as u8 (key_hi = key / nb <= 255 when nb >= 16843009)
	const uint32_t *bgrp;
	const uint8_t *keys8;
	//   bline[b]: one 64-byte line per bucket: u32 first item, u8 item count (255 = 255 or
	//            more), then the u8 keys of its first <= 59 items -- bounds and keys of a probe
	//            in ONE random line (replaces bgrp + keys8 when present)
	const uint4 *bline;
	//   bcode[b]: one 32-byte sector per bucket: u32 first item, u8 count (255 = not coded), the
	//            sorted key_hi multiset as a unary count code (build_bcode); replaces bline when
	//            the index's key_hi range is small (V = 0xffffffff / nb + 1 <= 80)
	const uint4 *bcode;
	//   khash: the probe records themselves, keyed by the full 32-bit key -- one 64-byte line
	//            per lookup: keys of 5 entries (0xffffffff = empty), their records (mid item,
	//            fwd | bwd << 16), an overflow word (continue at the next line).  Built when the
	//            bucket code does not apply (wide key_hi range: gapped indexes); the key
	//            0xffffffff itself lives in khash_ff = {present, mid, fwd | bwd << 16}
	const uint32_t *khash;
	const uint32_t *khash_ff;
	uint64_t khash_lines;
	int32_t khash_sec;        // 1: 32-byte sectors of 3 entries (8-bit run counts), 0: 64-byte lines
	//   ksorted: bit b set when bucket b's keys are non-decreasing as shorts (built with khash), so
	//            that its key-hash record is also prefill_votes's equal-key run (svg_probe_keys)
	const uint32_t *ksorted;
};

// ---------------------------------------------------------------------------------------------
// probe-image helpers shared by the vote path's probe kernels (svg_vote.hip) and the key
// lookups (svg_keys.hip)


// position (0..63) of the j-th (0-based) set bit of x; x has more than j set bits
__device__ __forceinline__ int select64(uint64_t x, int j)
{
	int pos = 0, c = __popc((uint32_t)x);
	if (j >= c) { j -= c; x >>= 32; pos = 32; }
	uint32_t v = (uint32_t)x;
	c = __popc(v & 0xffffu); if (j >= c) { j -= c; v >>= 16; pos += 16; }
	c = __popc(v & 0xffu); if (j >= c) { j -= c; v >>= 8; pos += 8; }
	c = __popc(v & 0xfu); if (j >= c) { j -= c; v >>= 4; pos += 4; }
	c = __popc(v & 0x3u); if (j >= c) { j -= c; v >>= 2; pos += 2; }
	return pos + (j >= (int)(v & 1u) ? 1 : 0);
}

// position of the j-th (0-based) zero bit at or above bit 40 of a 32-byte bucket code (LSB-first)
__device__ __forceinline__ int code_zero(const uint64_t z[4], int j)
{
	int base = 0;
#pragma unroll
	for (int q = 0; q < 4; q++) {
		const int c = __popcll(z[q]);
		if (j < c) return base + select64(z[q], j);
		j -= c;
		base += 64;
	}
	return 256;
}

// DevIndex::khash line of a key: the key scrambled by an odd constant (a bijection), reduced to
// [0, lines) by the high half of a 64-bit product
__device__ __forceinline__ uint64_t khash_line(uint32_t key, uint64_t lines)
{
	return ((uint64_t)(key * 0x9E3779B1u) * lines) >> 32;
}

// one 32-byte key-hash sector (3 entries: keys, midpoints, 8-bit run counts; the top half of the
// last word flags an overflow into the next sector): the key's record, or *more when the key may
// continue in the next sector
__device__ __forceinline__ bool khash_sector(const uint4 a, const uint4 b4, uint32_t key, uint2 &rec, bool &more)
{
	const uint32_t ks[3] = {a.x, a.y, a.z}, mid[3] = {a.w, b4.x, b4.y};
	const uint32_t fb[3] = {b4.z & 0xffffu, b4.z >> 16, b4.w & 0xffffu};
	bool found = false;
#pragma unroll
	for (int k = 0; k < 3; k++)
		if (ks[k] == key) { rec = make_uint2(mid[k], (fb[k] & 0xffu) | ((fb[k] >> 8) << 16)); found = true; }
	more = !found && (b4.w >> 16);
	return found;
}

// the probe record (mid item, fwd | bwd << 16) stored under key in DevIndex::khash, looked up from
// line L on; rec is left unchanged (and false returned) when the key has no record
__device__ __forceinline__ bool khash_find_from(const DevIndex &ix, uint32_t key, uint64_t L, uint2 &rec)
{
	bool found = false;
	if (ix.khash_sec) {
		for (;;) {
			const uint4 *l4 = (const uint4 *)(ix.khash + 8 * L);
			bool more;
			found = khash_sector(l4[0], l4[1], key, rec, more);
			if (!more) break;
			L = L + 1 == ix.khash_lines ? 0 : L + 1;
		}
	} else for (;;) {
		const uint4 *l4 = (const uint4 *)(ix.khash + 16 * L);
		const uint4 a = l4[0], b4 = l4[1], c4 = l4[2], d4 = l4[3];
		const uint32_t ks[5] = {a.x, a.y, a.z, a.w, b4.x};
		const uint32_t px[5] = {b4.y, b4.w, c4.y, c4.w, d4.y};
		const uint32_t py[5] = {b4.z, c4.x, c4.z, d4.x, d4.z};
#pragma unroll
		for (int k = 0; k < 5; k++)
			if (ks[k] == key) { rec = make_uint2(px[k], py[k]); found = true; }
		if (found || !d4.w) break;
		L = L + 1 == ix.khash_lines ? 0 : L + 1;
	}
	return found;
}

__device__ __forceinline__ bool khash_find(const DevIndex &ix, uint32_t key, uint2 &rec)
{
	if (key == 0xffffffffu) {
		if (!ix.khash_ff[0]) return false;
		rec = make_uint2(ix.khash_ff[1], ix.khash_ff[2]);
		return true;
	}
	return khash_find_from(ix, key, khash_line(key, ix.khash_lines), rec);
}

#define SVG_MAX_BLOCKS 64

struct svg_index {
	int device;
	hipStream_t stream;
	svg_host_index host;
	DevIndex dix;
	void *d_bstart, *d_keys, *d_vals, *d_values, *d_chr, *d_bgrp, *d_keys8, *d_bline, *d_bcode, *d_khash, *d_ksorted;
	uint32_t *d_scratch;
	size_t scratch_words;
	unsigned long long *d_stats;
	int stats_on;
	svg_batch_stats last_stats;
	uint64_t device_bytes;
	int n_cu;
	int wave_cap;   // > 0: blocks per CU cap of the wave kernel (set while it overlaps the probe kernel)
	int max_read_len;        // announced read-length bound (svg_set_max_read_length), picks the kernel variant
	// chunk pipeline: probe + lane kernels of chunk c run on the caller's stream while the wave
	// kernel of chunk c-1 runs on stream2, so the per-chunk buffers come in two slots (c & 1; three
	// with option host_slots 3)
	hipStream_t stream2;
	hipEvent_t ev_lane[3], ev_wave[3], ev_probe[3];   // slot's records + deferral list ready / wave kernel done / probe records ready
	void *d_prec[3]; size_t prec_cap[3];   // probe records of one chunk
	void *d_big[3]; size_t big_cap[3];     // probe_line_kernel's big-bucket list (count, slot indexes)
	// lane-per-read SE path (svg_lane.hip): candidate lists + deferral list, per-wave cold scratch
	void *d_lane[3]; size_t lane_cap[3];
	uint32_t *d_lscratch; size_t lscratch_words;     // light pass
	// svg_set_timing: event pairs per launch (kinds: 0 probe_kernel, 1 vote_kernel, 2 gather_kernel,
	// 3 lane_kernel), folded into the sums when the ring fills
	int timing;
	hipEvent_t tev[4][64][2];
	int tn[4], tcount[4];
	double tms[4];
	// staging for svg_vote_batch (host buffers): two sub-batch slots, uploads and downloads on
	// their own streams so PCIe traffic of sub-batches i+1 / i-1 overlaps the vote of i
	void *d_in[3]; size_t d_in_cap[3];     // uploads run one sub-batch ahead: three input slots
	void *d_out[3]; size_t d_out_cap[3];
	hipStream_t up_stream, down_stream;
	hipEvent_t ev_up[3], ev_done[3], ev_down[3];
	// sticky device error word (KParams::err) and the handle's last queued work: every call
	// orders its stream after the previous call's work, since both reuse the buffers above
	uint32_t *d_err;
	hipEvent_t ev_last;
	int last_pending;
	// host-buffer entry points (svg_io.hip): record compaction slots, pinned staging, worker pool
	struct svg_hostio *io;
	// multi-block indexes (<prefix>.NN.b.tab, NN = 00, 01, ...): this handle holds block 0; blocks
	// 1.. are handles of their own, voted after it in order with stored = 1
	int nblocks;
	struct svg_index *blk[SVG_MAX_BLOCKS];
	int stored;
	// svg_long_vote_batch's grow-only device arenas and pinned staging (svg_long.hip)
	struct svg_longws *lws;
};

#define HIPCHK(x) do { hipError_t _e = (x); if (_e != hipSuccess) { svg_set_error("HIP error %s at %s:%d", hipGetErrorString(_e), __FILE__, __LINE__); return SVG_E_DEVICE; } } while (0)

static inline int dmalloc(svg_index *h, void **p, size_t n)
{
	hipError_t e = hipMalloc(p, n ? n : 16);
	if (e != hipSuccess) { svg_set_error("hipMalloc(%zu) failed: %s", n, hipGetErrorString(e)); return SVG_E_NOMEM; }
	h->device_bytes += n;
	return 0;
}

int svg_index_finish_device(svg_index *h);

// grow-only device buffer
static inline int svg_ensure(svg_index *h, void **p, size_t *cap, size_t need)
{
	if (need <= *cap) return 0;
	hipFree(*p);
	*p = NULL;
	*cap = 0;
	if (dmalloc(h, p, need)) return SVG_E_NOMEM;
	*cap = need;
	return 0;
}

// svg_io.hip
void svg_io_free(svg_index *h);
// svg_long.hip
void svg_long_ws_free(svg_index *h);

// ---------------------------------------------------------------------------------------------
// kernel parameters (passed by value)
struct KParams {
	svg_params p;
	DevIndex ix;
	const char *seq1, *seq2;
	const uint64_t *off1, *off2;
	const uint16_t *len1, *len2;
	uint64_t n_reads;
	uint8_t *out;             // mapping records
	uint8_t *jout;            // subjunc records
	uint16_t *bm_out;
	uint32_t *scratch;        // per-wave cold state
	unsigned long long *stats; // probes, bucket_items, hits, results (may be NULL)
	int tol, ii_end;
	uint32_t low, high;
	const uint2 *precs;       // probe records of this chunk (probe_kernel)
	int nps;                  // probe slots per (end, strand) in precs
	uint32_t prec_stride;     // 0: records of read r at precs[r*per + i]; else SoA precs[i*stride + r]
	const uint32_t *idx;      // NULL: reads 0..n_reads-1; else the reads idx[0..*idx_count) (deferred by lane_kernel)
	const uint32_t *idx_count;
	uint32_t *work;           // indirect mode: zeroed work counter (waves grab deferred reads dynamically)
	int32_t static_eighths;   // indirect mode: eighths of the deferred reads dealt out statically
	int stored;               // records already hold earlier index blocks' results (multi-block, block > 0)
	uint32_t *err;            // sticky device error word (svg_device_status): bit 0 = a read needs more
	                          // probes than the announced read-length bound provides, bit 1 = a read
	                          // longer than the kernel variant's text buffer; such reads get zero records
};

// probe kernel parameters: one thread per (read, end, strand, subread x gap slot)
struct PParams {
	DevIndex ix;
	const char *seq1, *seq2;
	const uint64_t *off1, *off2;
	const uint16_t *len1, *len2;
	uint32_t n_reads;
	int nps;
	int total_subreads, reverse_r1, reverse_r2;
	uint64_t nb_magic;        // ceil(2^64 / nb): key / nb == umulhi64(key, nb_magic) for 32-bit keys
	uint2 *out;               // [read][end][strand][nps] (soa = 0) or [end][strand][nps][read] (soa = 1):
	                          // x = midpoint item, y = fwd | bwd << 16
	int soa;
	int window;               // one-shot bucket loads (keys of a bucket sorted as int16: nb >= 131073)
	int readmajor;            // soa output with read-major threads (consecutive threads = one read's probes)
	unsigned long long *stats;
	// 2-bit packed input (svg_packed_reads) per end, read r of the chunk at base
	// pk_starts[e][r] or pk_base0[e] + r * pk_stride[e]; seq/off unused when packed
	// bucket-line kernel: reads per LDS group; list of probes with > 59-item buckets
	uint32_t group;
	uint32_t *big_list, *big_count;   // [region][big_stride] slot indexes, [region] counts
	uint32_t big_stride, big_regions;
	int packed;
	const uint32_t *pk_bases[2], *pk_xmask[2];
	const uint64_t *pk_starts[2];
	uint64_t pk_stride[2], pk_base0[2];
};

// svg_vote.hip: a prepared batch (kernel parameters) and its per-chunk launch
struct VoteJob {
	KParams kp;
	PParams pp;
	int npmax, nps, ends;
	bool sj, lane, overlap_mode;
	uint64_t per_read, chunk;   // probe records per read; reads per chunk (<= 1 GiB of records)
};
int svg_vote_prepare(svg_index *h, const svg_params *p, const svg_reads *r1, const svg_reads *r2, svg_mapping_result *out,
                     svg_subjunc_result *jout, uint16_t *big_margin, VoteJob *job);
int svg_vote_chunk(svg_index *h, VoteJob *job, uint64_t c0, uint64_t cn, int slot, hipStream_t st, hipStream_t st2);
// the two halves of svg_vote_chunk: the probe kernels (into the slot's probe records), then the
// lane kernels on st and the wave kernel on st2
int svg_vote_chunk_probe(svg_index *h, VoteJob *job, uint64_t c0, uint64_t cn, int slot, hipStream_t st);
int svg_vote_chunk_vote(svg_index *h, VoteJob *job, uint64_t c0, uint64_t cn, int slot, hipStream_t st, hipStream_t st2);
int svg_vote_batch_device_packed(svg_index *h, const svg_params *p, const svg_reads *r1, const svg_reads *r2,
                                 const svg_packed_reads *pk, svg_mapping_result *out, svg_subjunc_result *jout,
                                 uint16_t *big_margin, hipStream_t stream);

// svg_lane.hip
int svg_lane_eligible(const svg_index *h, const svg_params *p, int paired, int sj);
// the parameter contract of every vote entry point (multi_best 1..3, top_scores 3, ...)
int svg_check_params(const svg_index *h, const svg_params *p, int paired);
int svg_lane_chunk(svg_index *h, int slot, const svg_params *p, const uint16_t *len, uint32_t n, const uint2 *precs,
                   int nps, uint8_t *out, uint8_t *jout, uint16_t *bm, const char *seq, const uint64_t *off,
                   unsigned long long *stats, uint32_t **defer_list, uint32_t **defer_count, hipStream_t st);
int svg_lane_pe_chunk(svg_index *h, int slot, const svg_params *p, const uint16_t *len1, const uint16_t *len2, uint32_t n,
                      const uint2 *precs, int nps, uint8_t *out, uint8_t *jout, uint16_t *bm_out, const char *seq1,
                      const uint64_t *off1, const char *seq2, const uint64_t *off2, unsigned long long *stats,
                      uint32_t **defer_list, uint32_t **defer_count, hipStream_t st);
int svg_timing_mark(svg_index *h, int k, int phase, hipStream_t st);

#endif
