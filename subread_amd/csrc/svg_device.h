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
};

struct svg_index {
	int device;
	hipStream_t stream;
	svg_host_index host;
	DevIndex dix;
	void *d_bstart, *d_keys, *d_vals, *d_values, *d_chr, *d_bgrp, *d_keys8, *d_bline;
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
	// kernel of chunk c-1 runs on stream2, so the per-chunk buffers come in two slots (c & 1)
	hipStream_t stream2;
	hipEvent_t ev_lane[2], ev_wave[2];   // slot's records + deferral list ready / wave kernel done
	void *d_prec[2]; size_t prec_cap[2];   // probe records of one chunk
	// lane-per-read SE path (svg_lane.hip): candidate lists + deferral list, per-wave cold scratch
	void *d_lane[2]; size_t lane_cap[2];
	uint32_t *d_lscratch; size_t lscratch_words;     // light pass
	uint32_t *d_lscratch2; size_t lscratch2_words;   // heavy pass
	// svg_set_timing: event pairs per launch (kinds: 0 probe_kernel, 1 vote_kernel, 2 gather_kernel,
	// 3 lane_kernel), folded into the sums when the ring fills
	int timing;
	hipEvent_t tev[4][64][2];
	int tn[4], tcount[4];
	double tms[4];
	// staging for svg_vote_batch (host buffers): two sub-batch slots, uploads and downloads on
	// their own streams so PCIe traffic of sub-batches i+1 / i-1 overlaps the vote of i
	void *d_in[2]; size_t d_in_cap[2];
	void *d_out[2]; size_t d_out_cap[2];
	hipStream_t up_stream, down_stream;
	hipEvent_t ev_up[2], ev_done[2], ev_down[2];
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

// svg_lane.hip
int svg_lane_eligible(const svg_index *h, const svg_params *p, int paired, int sj);
int svg_lane_chunk(svg_index *h, int slot, const svg_params *p, const uint16_t *len, uint32_t n, const uint2 *precs,
                   int nps, uint8_t *out, uint8_t *jout, uint16_t *bm, unsigned long long *stats, uint32_t **defer_list,
                   uint32_t **defer_count, hipStream_t st);
int svg_lane_pe_chunk(svg_index *h, int slot, const svg_params *p, const uint16_t *len1, const uint16_t *len2, uint32_t n,
                      const uint2 *precs, int nps, uint8_t *out, unsigned long long *stats, uint32_t **defer_list,
                      uint32_t **defer_count, hipStream_t st);
int svg_timing_mark(svg_index *h, int k, int phase, hipStream_t st);

#endif
