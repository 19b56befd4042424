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
};

struct svg_index {
	int device;
	hipStream_t stream;
	svg_host_index host;
	DevIndex dix;
	void *d_bstart, *d_keys, *d_vals, *d_values, *d_chr;
	uint32_t *d_scratch;
	size_t scratch_words;
	unsigned long long *d_stats;
	int stats_on;
	svg_batch_stats last_stats;
	uint64_t device_bytes;
	int n_cu;
	int max_read_len;        // announced read-length bound (svg_set_max_read_length), picks the kernel variant
	void *d_prec; size_t prec_cap;   // probe records of one chunk
	// svg_set_timing: event pairs per launch, folded into the sums when the ring fills
	int timing;
	hipEvent_t tev[2][64][2];
	int tn[2], tcount[2];
	double tms[2];
	// staging for svg_vote_batch (host buffers)
	void *d_in; size_t d_in_cap;
	void *d_out; size_t d_out_cap;
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

#endif
