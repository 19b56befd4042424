// svg_keys.hip -- equal-key runs of arbitrary subread keys (include/subread_vote.h svg_probe_keys*).
//
// cellCounts does not call gehash_go_X: its voting first lists, for every subread of a read,
// the bucket-local run of items whose key equals the subread's (prefill_votes,
// cell-counts.c:432-491), and votes over those lists itself.  That lookup is the probe half of
// the vote path (a3-a4) with a different widening: binary search of (short)(key / buckets) in
// the bucket's keys (sorted-hashtable.c's layout), then forward / backward steps of imax/4,
// /3, /3 ... that only land on equal keys, then single steps to the run's ends.  One thread
// per key runs exactly that (the literal steps matter for small indexes, whose bucket keys are
// not sorted as shorts); every image the vote path builds for its own probes is bypassed,
// since the plain bounds + i16 keys are always resident.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "subread_vote.h"
#include "svg_internal.h"
#include "svg_device.h"

struct KeyParams {
	const uint32_t *bstart;
	const int16_t *keys;
	uint32_t nb;
	const uint32_t *in;
	uint64_t n;
	uint32_t *first, *count;
};

__global__ void __launch_bounds__(256) probe_keys_kernel(KeyParams kp)
{
	for (uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x; t < kp.n; t += (uint64_t)gridDim.x * 256u) {
		const uint32_t sub = kp.in[t];
		const uint32_t b = sub % kp.nb;
		const uint32_t base = kp.bstart[b];
		const int items = (int)(kp.bstart[b + 1] - base);
		const int16_t *ck = kp.keys + base;
		const int16_t key = (int16_t)(sub / kp.nb);
		uint32_t f = 0, c = 0;
		if (items > 0) {
			int imin = 0, imax = items - 1, last;
			bool found = true;
			for (;;) {
				last = (imin + imax) / 2;
				const int16_t cur = ck[last];
				if (cur > key) imax = last - 1;
				else if (cur < key) imin = last + 1;
				else break;
				if (imax < imin) { found = false; break; }
			}
			if (found) {
				imax -= imin;
				const int start = last;
				int stoploc;
				for (int step = imax / 4; step > 1; step /= 3)
					for (;;) {
						const int tl = last + step;
						if (tl >= items || ck[tl] != key) break;
						last = tl;
					}
				for (;;) {
					last++;
					if (last == items || ck[last] != key) { stoploc = last; last = start; break; }
				}
				for (int step = imax / 4; step > 1; step /= 3)
					for (;;) {
						const int tl = last - step;
						if (tl < imin || ck[tl] != key) break;
						last = tl;
					}
				while (!(last == imin || ck[last - 1] != key)) last--;
				f = (uint32_t)last;
				c = (uint32_t)(stoploc - last);
			}
		}
		kp.first[t] = f;
		kp.count[t] = c;
	}
}

static svg_index *key_block(svg_index *h, int block)
{
	if (!h) { svg_set_error("svg_probe_keys: no index"); return NULL; }
	if (block < 0 || block >= (h->nblocks > 0 ? h->nblocks : 1)) {
		svg_set_error("svg_probe_keys: block %d of an index with %d block(s)", block, h->nblocks > 0 ? h->nblocks : 1);
		return NULL;
	}
	return block ? h->blk[block] : h;
}

static int launch_keys(svg_index *h, svg_index *bk, const uint32_t *keys, uint64_t n, uint32_t *first, uint32_t *count,
                       hipStream_t st)
{
	if (n == 0) return 0;
	KeyParams kp;
	kp.bstart = bk->dix.bstart;
	kp.keys = bk->dix.keys;
	kp.nb = bk->dix.nb;
	kp.in = keys;
	kp.n = n;
	kp.first = first;
	kp.count = count;
	uint64_t blocks = (n + 255) / 256, bmax = (uint64_t)h->n_cu * 16;
	if (blocks > bmax) blocks = bmax;
	hipLaunchKernelGGL(probe_keys_kernel, dim3((unsigned)blocks), dim3(256), 0, st, kp);
	HIPCHK(hipGetLastError());
	return 0;
}

extern "C" int svg_probe_keys_device(svg_index *h, int block, const uint32_t *keys, uint64_t n, uint32_t *first,
                                     uint32_t *count, void *hip_stream)
{
	svg_index *bk = key_block(h, block);
	if (!bk) return SVG_E_ARG;
	if (n && (!keys || !first || !count)) { svg_set_error("svg_probe_keys_device: NULL buffer"); return SVG_E_ARG; }
	HIPCHK(hipSetDevice(h->device));
	hipStream_t st = hip_stream ? (hipStream_t)hip_stream : h->stream;
	// the handle's earlier work first (its buffers are not touched, but the index may still be
	// under construction on the handle's stream)
	if (st != h->stream) {
		hipEvent_t ev;
		HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
		HIPCHK(hipEventRecord(ev, h->stream));
		HIPCHK(hipStreamWaitEvent(st, ev, 0));
		HIPCHK(hipEventDestroy(ev));
	}
	return launch_keys(h, bk, keys, n, first, count, st);
}

extern "C" int svg_probe_keys(svg_index *h, int block, const uint32_t *keys, uint64_t n, uint32_t *first, uint32_t *count)
{
	svg_index *bk = key_block(h, block);
	if (!bk) return SVG_E_ARG;
	if (n == 0) return 0;
	if (!keys || !first || !count) { svg_set_error("svg_probe_keys: NULL buffer"); return SVG_E_ARG; }
	HIPCHK(hipSetDevice(h->device));
	const uint64_t CH = 16u << 20;   // keys per round trip (192 MB of device buffers)
	const uint64_t m = n < CH ? n : CH;
	void *d = NULL;
	if (dmalloc(h, &d, 12 * m)) return SVG_E_NOMEM;
	uint32_t *dk = (uint32_t *)d, *df = dk + m, *dc = df + m;
	int rc = 0;
	for (uint64_t o = 0; o < n && !rc; o += m) {
		const uint64_t k = n - o < m ? n - o : m;
		if (hipMemcpyAsync(dk, keys + o, 4 * k, hipMemcpyHostToDevice, h->stream) != hipSuccess) { rc = SVG_E_DEVICE; break; }
		if ((rc = launch_keys(h, bk, dk, k, df, dc, h->stream))) break;
		if (hipMemcpyAsync(first + o, df, 4 * k, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
		    hipMemcpyAsync(count + o, dc, 4 * k, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
		    hipStreamSynchronize(h->stream) != hipSuccess) { rc = SVG_E_DEVICE; break; }
	}
	if (rc == SVG_E_DEVICE) svg_set_error("svg_probe_keys: HIP error %s", hipGetErrorString(hipGetLastError()));
	hipFree(d);
	h->device_bytes -= 12 * m;
	return rc;
}
