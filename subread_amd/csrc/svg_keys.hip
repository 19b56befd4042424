// svg_keys.hip -- equal-key runs of arbitrary subread keys (include/subread_vote.h svg_probe_keys*).
//
// cellCounts does not call gehash_go_X: its voting first lists, for every subread of a read,
// the bucket-local run of items whose key equals the subread's (prefill_votes,
// cell-counts.c:432-491), and votes over those lists itself.  That lookup is the probe half of
// the vote path (a3-a4) with a different widening: binary search of (short)(key / buckets) in
// the bucket's keys (sorted-hashtable.c's layout), then forward / backward steps of imax/4,
// /3, /3 ... that only land on equal keys, then single steps to the run's ends.
//
// In a bucket whose keys are sorted, those steps find exactly the whole equal-key run -- the
// run the vote path's probe images already hold:
//   bucket code (full indexes, build_bcode): one random 32-byte sector per key gives the run's
//     bucket-local bounds directly (count byte 255 = not coded: unsorted or > 169 items);
//   key hash (gapped / small indexes, build_khash): one random sector gives the record
//     (mid item, fwd, bwd) of the run, and the bucket's first item turns it bucket-local; a
//     bucket whose keys are not sorted (DevIndex::ksorted) takes the literal search instead.
// The literal search (one thread per key over the resident bounds + i16 keys) answers
// everything else; SVG_KEYS_LITERAL=1 forces it (A/B and tests).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "subread_vote.h"
#include "svg_internal.h"
#include "svg_device.h"

struct KeyParams {
	DevIndex ix;
	const uint32_t *bstart;
	const int16_t *keys;
	uint32_t nb;
	const uint32_t *in;
	uint64_t n;
	uint32_t *first, *count;
};

// prefill_votes's search, literally (cell-counts.c:432-491)
__device__ __forceinline__ void keys_literal(const KeyParams &kp, uint32_t sub, uint32_t b, uint32_t &f, uint32_t &c)
{
	{
		const uint32_t base = kp.bstart[b];
		const int items = (int)(kp.bstart[b + 1] - base);
		const int16_t *ck = kp.keys + base;
		const int16_t key = (int16_t)(sub / kp.nb);
		f = 0;
		c = 0;
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
	}
}

#define KEYS_LITERAL 0
#define KEYS_CODE    1
#define KEYS_KHASH   2
template <int IMG>
__global__ void __launch_bounds__(256) probe_keys_kernel(KeyParams kp)
{
	for (uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x; t < kp.n; t += (uint64_t)gridDim.x * 256u) {
		const uint32_t sub = kp.in[t];
		const uint32_t q = sub / kp.nb, b = sub - q * kp.nb;
		uint32_t f = 0, c = 0;
		bool literal = IMG == KEYS_LITERAL;
		if (IMG == KEYS_CODE) {
			// the bucket's 32-byte code: the run of key_hi = q is [fe, ee) of the bucket's items
			const uint4 *c4 = kp.ix.bcode + 2 * (size_t)b;
			const uint4 u0 = c4[0], u1 = c4[1];
			const uint32_t n = u0.y & 255u;
			literal = n == 255u;
			if (!literal && n) {
				const uint64_t z[4] = {~(((uint64_t)u0.y << 32) | u0.x) & ~0xffffffffffull, ~(((uint64_t)u0.w << 32) | u0.z),
				                       ~(((uint64_t)u1.y << 32) | u1.x), ~(((uint64_t)u1.w << 32) | u1.z)};
				const int k = (int)q;
				const int fe = k ? code_zero(z, k - 1) - 40 - (k - 1) : 0;
				const int ee = code_zero(z, k) - 40 - k;
				if (ee > fe) { f = (uint32_t)fe; c = (uint32_t)(ee - fe); }
			}
		} else if (IMG == KEYS_KHASH) {
			// (the image keys a run by (u16)key_hi * nb + bucket: quotients past 16 bits, which only
			// tiny indexes have, compare as wrapped shorts in the reference -- literal search)
			literal = q > 0xffffu || !((kp.ix.ksorted[b >> 5] >> (b & 31u)) & 1u);
			if (!literal) {
				uint2 rec;
				if (khash_find(kp.ix, sub, rec)) {
					{
						const uint32_t fwd = rec.y & 0xffffu, bwd = rec.y >> 16;
						f = rec.x - bwd - kp.bstart[b];
						c = fwd + bwd;
					}
				}
			}
		}
		if (literal) keys_literal(kp, sub, b, f, c);
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
	kp.ix = bk->dix;
	kp.bstart = bk->dix.bstart;
	kp.keys = bk->dix.keys;
	kp.nb = bk->dix.nb;
	kp.in = keys;
	kp.n = n;
	kp.first = first;
	kp.count = count;
	uint64_t blocks = (n + 255) / 256, bmax = (uint64_t)h->n_cu * 16;
	if (blocks > bmax) blocks = bmax;
	const bool lit = svg_get_option("keys_literal") != 0;
	if (!lit && bk->dix.bcode) hipLaunchKernelGGL(probe_keys_kernel<KEYS_CODE>, dim3((unsigned)blocks), dim3(256), 0, st, kp);
	else if (!lit && bk->dix.khash && bk->dix.ksorted)
		hipLaunchKernelGGL(probe_keys_kernel<KEYS_KHASH>, dim3((unsigned)blocks), dim3(256), 0, st, kp);
	else hipLaunchKernelGGL(probe_keys_kernel<KEYS_LITERAL>, dim3((unsigned)blocks), dim3(256), 0, st, kp);
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
