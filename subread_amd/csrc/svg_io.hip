// svg_io.hip -- host-buffer entry points of the vote path (include/subread_vote.h):
//
//   * 2-bit packed reads: svg_pack_reads packs ASCII reads on the host,
//     unpack_reads restores, in HBM, exactly the characters every kernel's arithmetic can
//     tell apart, so the vote kernels are the same for both input forms;
//   * record compaction for the device-to-host copy: ~1.2 of a read end's 3 mapping_result_t
//     are non-zero, so compact_records ships only those (plus one flag byte per read) and the
//     host writes the caller's full records (copy or zero) in worker threads;
//   * the sub-batch pipeline behind svg_vote_batch / svg_vote_batch_packed: upload of
//     sub-batch i+1, vote + compaction of i, download of i-2 and host expansion of i-3 all
//     overlap (PCIe in, GPU, PCIe out and host memory bandwidth are separate resources).
//
// The reference hands reads to do_voting through fetch_next_read_pair (core.c:1121-1211)
// and reads the bigtable it writes (core-bigtable.c:84-131); see INTEGRATION.md.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>
#include <stdio.h>
#include <thread>
#include <mutex>
#include <condition_variable>
#include <deque>
#include <functional>
#include <vector>
#include <chrono>
#include <emmintrin.h>
#include <sched.h>
#include <ctype.h>
#include <pthread.h>
#include <unistd.h>
#include <sys/syscall.h>
#include "subread_vote.h"
#include "svg_internal.h"
#include "svg_device.h"

// ============================================================================ packed reads
// base2int (subread.h:238): A=0 G=1 C=2 T=3, any other character 2 below 'G' and 3 above.
static inline uint32_t pack_code(unsigned char c) { return c < 'G' ? (c == 'A' ? 0u : 2u) : (c == 'G' ? 1u : 3u); }
// Characters that are not A/C/G/T/U: reverse_read's table (input-files.c:1111) turns them
// into 'N'; 'U' complements to 'A' like 'T' and is T in every other use as well.
static inline bool pack_exception(unsigned char c) { return !(c == 'A' || c == 'C' || c == 'G' || c == 'T' || c == 'U'); }

// One thread per output dword of the ASCII text (4 bases).  An exception base becomes '.'
// (code 2) or 'N' (code 3): both pack to the same key codes as the original character
// (genekey2int), both complement to 'N', and both take the default branch of match_chro's
// forward comparison (gene-value-index.c:911-929) -- so every kernel sees the same read.
struct UnpackParams {
	const uint32_t *bases, *xmask;
	const uint64_t *starts;
	uint64_t stride, base0;   // without starts: read r starts at base base0 + r * stride
	const uint16_t *lens;
	uint32_t n, S;            // reads, text bytes per read (multiple of 4)
	uint32_t *text;
	uint64_t *offs;
	uint32_t *err;
};

__global__ void __launch_bounds__(256) unpack_reads(UnpackParams u)
{
	const uint32_t W = u.S >> 2;
	const uint64_t total = (uint64_t)u.n * W;
	for (uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x; t < total; t += (uint64_t)gridDim.x * 256u) {
		const uint32_t r = (uint32_t)(t / W), w = (uint32_t)(t - (uint64_t)r * W);
		int len = u.lens[r];
		if (len > SVG_READ_KEEP) len = SVG_READ_KEEP;
		if (!u.starts && (uint64_t)len > u.stride) len = (int)u.stride;   // contract: lens[r] <= stride
		if (w == 0) {
			u.offs[r] = (uint64_t)r * u.S;
			if ((uint32_t)len > u.S) atomicOr(u.err, 1u);   // beyond the announced read-length bound
		}
		uint32_t o = 0;
		if (4 * (int)w < len) {
			const uint64_t k0 = (u.starts ? u.starts[r] : u.base0 + (uint64_t)r * u.stride) + 4u * w;
#pragma unroll
			for (int j = 0; j < 4; j++) {
				if (4 * (int)w + j >= len) break;
				const uint64_t k = k0 + (uint64_t)j;
				const uint32_t code = (u.bases[k >> 4] >> (30u - 2u * (uint32_t)(k & 15u))) & 3u;
				const uint32_t x = u.xmask ? (u.xmask[k >> 5] >> (31u - (uint32_t)(k & 31u))) & 1u : 0u;
				const uint32_t c = x ? (code == 2u ? '.' : 'N') : ((0x54434741u >> (8u * code)) & 0xffu);   // "AGCT"
				o |= c << (8 * j);
			}
		}
		u.text[t] = o;
	}
}

// 16-byte streaming stores of n bytes (dst and n 16-byte aligned, src 16-byte aligned)
static inline void stream_out(uint8_t *dst, const uint8_t *src, size_t n)
{
	for (size_t i = 0; i < n; i += 16)
		_mm_stream_si128((__m128i *)(dst + i), _mm_load_si128((const __m128i *)(src + i)));
}

// ============================================================================ record compaction
// One wave per tile of 64 reads: the tile's records (R per read, RW dwords each) are staged in
// LDS with coalesced loads, each lane flags its read's non-zero records, a wave scan places
// them, one atomic per tile reserves the tile's range of the compact array, and the compacted
// tile leaves in coalesced stores.  flags[r] bit k = record k of read r is non-zero;
// tile_base[t] = first compact record of tile t (tiles are placed in atomic order).
template <int RW>
__global__ void __launch_bounds__(64) compact_records(const uint32_t *src, int R, uint32_t m, uint32_t *dst, uint8_t *flags,
                                                      uint32_t *tile_base, uint32_t *counter)
{
	extern __shared__ uint32_t sm[];
	const int lane = threadIdx.x;
	const uint32_t r0 = blockIdx.x * 64u;
	const int nr = m - r0 < 64u ? (int)(m - r0) : 64;
	const int per = R * RW;
	const uint32_t *s = src + (size_t)r0 * per;
	for (int i = lane; i < nr * per; i += 64) sm[i] = s[i];
	__syncthreads();
	uint32_t f = 0;
	int c = 0;
	if (lane < nr) {
		for (int k = 0; k < R; k++) {
			uint32_t nz = 0;
#pragma unroll
			for (int d = 0; d < RW; d++) nz |= sm[(lane * R + k) * RW + d];
			if (nz) { f |= 1u << k; c++; }
		}
	}
	int incl = c;
	for (int o = 1; o < 64; o <<= 1) {
		const int t = __shfl_up(incl, o);
		if (lane >= o) incl += t;
	}
	const int total = __shfl(incl, 63), excl = incl - c;
	uint32_t base = 0;
	if (lane == 0) {
		base = atomicAdd(counter, (uint32_t)total);
		tile_base[blockIdx.x] = base;
	}
	base = __shfl(base, 0);
	if (lane < nr) flags[r0 + lane] = (uint8_t)f;
	uint32_t *o = sm + 64 * per;
	int j = excl;
	for (int k = 0; k < R; k++)
		if ((f >> k) & 1u) {
#pragma unroll
			for (int d = 0; d < RW; d++) o[j * RW + d] = sm[(lane * R + k) * RW + d];
			j++;
		}
	__syncthreads();
	for (int i = lane; i < total * RW; i += 64) dst[(size_t)base * RW + i] = o[i];
}

// ============================================================================ worker pool
// A few host threads for the record expansion; jobs carry a group (the staging slot) so the
// pipeline can wait for one slot's expansion before reusing its buffer.
struct SvgPool {
	std::vector<std::thread> th;
	std::mutex mu;
	std::condition_variable cv, cv_done;
	std::deque<std::pair<int, std::function<void()>>> q;
	int pending[4] = {0, 0, 0, 0};
	bool stop = false;

	explicit SvgPool(int n, const cpu_set_t *cpus = NULL)
	{
		for (int i = 0; i < n; i++) {
			th.emplace_back([this] {
				for (;;) {
					std::pair<int, std::function<void()>> job;
					{
						std::unique_lock<std::mutex> lk(mu);
						cv.wait(lk, [this] { return stop || !q.empty(); });
						if (q.empty()) return;
						job = std::move(q.front());
						q.pop_front();
					}
					job.second();
					std::lock_guard<std::mutex> lk(mu);
					if (--pending[job.first] == 0) cv_done.notify_all();
				}
			});
			// expansion workers on the CPUs of the GPU's NUMA node (svg_host_placement)
			if (cpus) pthread_setaffinity_np(th.back().native_handle(), sizeof(cpu_set_t), cpus);
		}
	}
	~SvgPool()
	{
		{
			std::lock_guard<std::mutex> lk(mu);
			stop = true;
		}
		cv.notify_all();
		for (auto &t : th) t.join();
	}
	void post(int g, std::function<void()> fn)
	{
		{
			std::lock_guard<std::mutex> lk(mu);
			pending[g]++;
			q.emplace_back(g, std::move(fn));
		}
		cv.notify_one();
	}
	void wait(int g)
	{
		std::unique_lock<std::mutex> lk(mu);
		cv_done.wait(lk, [&] { return pending[g] == 0; });
	}
};

// CPUs this process may run on: its affinity mask, capped by a cgroup CPU quota (v2 cpu.max or
// v1 cfs_quota/cfs_period) -- hardware_concurrency() reports the whole machine (256 on the
// GPU boxes, of which a 1-GPU job gets 16)
static int usable_cpus()
{
	int n = 0;
	cpu_set_t cs;
	if (sched_getaffinity(0, sizeof cs, &cs) == 0) n = CPU_COUNT(&cs);
	if (n <= 0) n = (int)std::thread::hardware_concurrency();
	if (n <= 0) n = 4;
	long quota = -1, period = 0;
	if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
		char q[32];
		if (fscanf(f, "%31s %ld", q, &period) == 2 && strcmp(q, "max") != 0) quota = atol(q);
		fclose(f);
	} else if (FILE *f1 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
		if (fscanf(f1, "%ld", &quota) != 1) quota = -1;
		fclose(f1);
		if (FILE *f2 = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
			if (fscanf(f2, "%ld", &period) != 1) period = 0;
			fclose(f2);
		}
	}
	if (quota > 0 && period > 0) {
		int c = (int)(quota / period);
		if (c < 1) c = 1;
		if (c < n) n = c;
	}
	return n;
}

// expansion workers of one handle: SVG_HOST_THREADS, else this rank's share of the usable CPUs
// (one rank per GPU: LOCAL_WORLD_SIZE ranks share the node's CPUs), at most 12 -- measured at
// C3 on one box in one call (profiles/r02_host_variance/ab_threads_*.log): 8 threads 371.7 /
// 264.8, 12 threads 399.1 / 402.2, 16 threads 399.8 / 383.7 Mreads/s -- and at least 2
static int host_threads()
{
	const int64_t o = svg_get_option("host_threads");
	if (o > 0) return (int)o;
	int n = usable_cpus();
	const char *lw = getenv("LOCAL_WORLD_SIZE");
	int ranks = lw ? atoi(lw) : 1;
	if (ranks > 1) n /= ranks;
	if (n < 2) n = 2;
	return n < 12 ? n : 12;
}

extern "C" int svg_host_threads(void) { return host_threads(); }

// ============================================================================ NUMA placement
// Each rank's host side -- the expansion workers that write 204 B per read into the caller's
// records, the pinned staging of the compacted downloads, and (through svg_host_alloc) the caller's
// own pinned reads and records -- belongs on the NUMA node of its GPU's PCIe root: at 8 ranks the
// node's memory system carries ~90 GB/s of writes per rank.

// "0-15,64-79" -> set bits (at most max), count
extern "C" int svg_cpulist_parse(const char *list, uint8_t *mask, int max)
{
	int n = 0;
	const char *p = list;
	while (p && *p) {
		while (*p == ',' || isspace((unsigned char)*p)) p++;
		if (!isdigit((unsigned char)*p)) break;
		long a = strtol(p, (char **)&p, 10), b = a;
		if (*p == '-') b = strtol(p + 1, (char **)&p, 10);
		for (long c = a; c <= b && c < max; c++)
			if (c >= 0 && !mask[c]) { mask[c] = 1; n++; }
	}
	return n;
}

static int read_small(const char *path, char *buf, int cap)
{
	FILE *f = fopen(path, "r");
	if (!f) return -1;
	int n = (int)fread(buf, 1, (size_t)cap - 1, f);
	fclose(f);
	buf[n > 0 ? n : 0] = 0;
	return n;
}

// the NUMA node of a HIP device's PCIe function (sysfs), -1 if unknown
static int device_numa_node(int device)
{
	char bus[64], path[256], buf[64];
	if (hipDeviceGetPCIBusId(bus, sizeof bus, device) != hipSuccess) { (void)hipGetLastError(); return -1; }
	for (char *c = bus; *c; c++) *c = (char)tolower((unsigned char)*c);
	snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
	if (read_small(path, buf, sizeof buf) <= 0) return -1;
	return atoi(buf);
}

// CPUs of node `node` this process may run on (affinity mask), as a cpu_set_t; returns the count
static int node_cpus(int node, cpu_set_t *out)
{
	CPU_ZERO(out);
	if (node < 0) return 0;
	char path[128], buf[4096];
	snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
	if (read_small(path, buf, sizeof buf) <= 0) return 0;
	static uint8_t m[CPU_SETSIZE];
	memset(m, 0, sizeof m);
	svg_cpulist_parse(buf, m, CPU_SETSIZE);
	cpu_set_t aff;
	if (sched_getaffinity(0, sizeof aff, &aff)) return 0;
	int n = 0;
	for (int c = 0; c < CPU_SETSIZE; c++)
		if (m[c] && CPU_ISSET(c, &aff)) { CPU_SET(c, out); n++; }
	return n;
}

// the placement of device `device`'s host side: node, and the usable CPUs on it
struct HostPlacement { int node, ncpus; cpu_set_t cpus; };
static HostPlacement placement_of(int device)
{
	HostPlacement hp;
	hp.node = device_numa_node(device);
	hp.ncpus = node_cpus(hp.node, &hp.cpus);
	return hp;
}

extern "C" int svg_host_placement(int device, int *node, int *cpus_on_node)
{
	HostPlacement hp = placement_of(device);
	if (node) *node = hp.node;
	if (cpus_on_node) *cpus_on_node = hp.ncpus;
	return 0;
}

#ifndef MPOL_DEFAULT
#define MPOL_DEFAULT 0
#define MPOL_PREFERRED 1
#endif

// pinned host memory whose pages come from `node` (hipHostMallocNumaUser: the allocation follows
// the calling thread's memory policy, set to "preferred: node" around the call and restored)
static hipError_t host_malloc_on(void **p, size_t n, int node)
{
	if (node < 0 || node >= 1024) return hipHostMalloc(p, n, hipHostMallocDefault);
	unsigned long oldmask[16], mask[16];
	int oldmode = MPOL_DEFAULT;
	memset(oldmask, 0, sizeof oldmask);
	memset(mask, 0, sizeof mask);
	const bool have_old = syscall(SYS_get_mempolicy, &oldmode, oldmask, 1024ul, (void *)0, 0ul) == 0;
	mask[node / 64] |= 1ul << (node % 64);
	const bool set = syscall(SYS_set_mempolicy, MPOL_PREFERRED, mask, 1024ul) == 0;
	hipError_t e = hipHostMalloc(p, n, set ? (hipHostMallocDefault | hipHostMallocNumaUser) : hipHostMallocDefault);
	if (set) {
		if (have_old) syscall(SYS_set_mempolicy, oldmode, oldmode == MPOL_DEFAULT ? (unsigned long *)0 : oldmask, 1024ul);
		else syscall(SYS_set_mempolicy, MPOL_DEFAULT, (unsigned long *)0, 0ul);
	}
	return e;
}

extern "C" int svg_host_alloc(svg_index *h, size_t bytes, void **out)
{
	if (!h || !out) { svg_set_error("svg_host_alloc: NULL argument"); return SVG_E_ARG; }
	*out = NULL;
	const int node = device_numa_node(h->device);
	if (host_malloc_on(out, bytes ? bytes : 1, node) != hipSuccess) {
		(void)hipGetLastError();
		*out = NULL;
		svg_set_error("svg_host_alloc: %zu pinned bytes failed", bytes);
		return SVG_E_NOMEM;
	}
	return 0;
}

extern "C" void svg_host_free(void *p)
{
	if (p) hipHostFree(p);
}

// ============================================================================ per-handle state
struct svg_hostio {
	SvgPool *pool;
	uint32_t *d_cnt;                         // [slot][4]: compact mapping / subjunc record counts
	void *d_text[3]; size_t d_text_cap[3];   // unpacked reads (packed input), per device slot
	void *d_offs[3]; size_t d_offs_cap[3];
	void *d_comp[3]; size_t d_comp_cap[3];   // compacted sub-batch (same layout as a staging slot)
	uint32_t *h_cnt;                         // pinned [slot][4] (3 slots): compact record counts
	uint8_t *h_stage[3]; size_t h_stage_cap[3];   // pinned host staging of compacted sub-batches
	int node;                                // NUMA node of the GPU (-1 unknown): staging pages, workers
	int node_cpus;                           // usable CPUs on it (0: workers are not pinned)
	cpu_set_t cpus;
};

void svg_io_free(svg_index *h)
{
	svg_hostio *io = h->io;
	if (!io) return;
	delete io->pool;
	hipFree(io->d_cnt);
	for (int s = 0; s < 3; s++) {
		hipFree(io->d_text[s]);
		hipFree(io->d_offs[s]);
	}
	for (int s = 0; s < 3; s++) {
		hipFree(io->d_comp[s]);
		hipHostFree(io->h_stage[s]);
	}
	hipHostFree(io->h_cnt);
	free(io);
	h->io = NULL;
}

static int io_get(svg_index *h, svg_hostio **out)
{
	if (!h->io) {
		svg_hostio *io = (svg_hostio *)calloc(1, sizeof(svg_hostio));
		if (!io) { svg_set_error("out of host memory"); return SVG_E_NOMEM; }
		h->io = io;
		HostPlacement hp = placement_of(h->device);
		io->node = hp.node;
		io->node_cpus = hp.ncpus;
		io->cpus = hp.cpus;
		int rc;
		if ((rc = dmalloc(h, (void **)&io->d_cnt, 64))) return rc;
		HIPCHK(hipHostMalloc((void **)&io->h_cnt, 64, hipHostMallocDefault));
	}
	*out = h->io;
	return 0;
}

static int host_ensure(void **p, size_t *cap, size_t need, int node)
{
	if (need <= *cap) return 0;
	hipHostFree(*p);
	*p = NULL;
	*cap = 0;
	if (host_malloc_on(p, need, node) != hipSuccess) {
		(void)hipGetLastError();
		svg_set_error("hipHostMalloc(%zu) failed", need);
		return SVG_E_NOMEM;
	}
	*cap = need;
	return 0;
}

// layout of one compacted sub-batch (device slot and host staging slot alike)
struct CompLayout {
	size_t o_flags, o_tile, o_rec, o_jflags, o_jtile, o_jrec, o_bm, bytes;
	uint32_t tiles;
};

static CompLayout comp_layout(uint64_t m, int R, int ends, bool jo, bool bmo)
{
	CompLayout L;
	auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
	L.tiles = (uint32_t)((m + 63) / 64);
	L.o_flags = 0;
	L.o_tile = al(m);
	L.o_rec = al(L.o_tile + 4 * (size_t)L.tiles);
	size_t e = al(L.o_rec + m * R * 68);
	L.o_jflags = L.o_jtile = L.o_jrec = e;
	if (jo) {
		L.o_jflags = e;
		L.o_jtile = al(e + m);
		L.o_jrec = al(L.o_jtile + 4 * (size_t)L.tiles);
		e = al(L.o_jrec + m * R * 16);
	}
	L.o_bm = e;
	if (bmo) e = al(e + m * ends * SVG_BIG_MARGIN_WORDS * 2);
	L.bytes = e;
	return L;
}

// the largest read length of reads [b, b+m) (truncated like read_line) and the per-length
// check that every kept length fits the kernels' 192 probes per strand
static int sub_max_len(const svg_index *h, const svg_params *p, const uint16_t *l1, const uint16_t *l2, uint64_t b,
                       uint64_t m, int *out)
{
	int mx = 16;
	for (int e = 0; e < (l2 ? 2 : 1); e++) {
		const uint16_t *ln = (e ? l2 : l1) + b;
		int v = 0;
		for (uint64_t i = 0; i < m; i++) v = ln[i] > v ? ln[i] : v;
		if (v > mx) mx = v;
	}
	if (mx > SVG_READ_KEEP) mx = SVG_READ_KEEP;
	const int gap = h->dix.gap;
	for (int len = 15 + gap; len <= mx; len++) {
		int cr = (len - 15 - gap) << 16, step;
		if (len <= 160) { step = cr / (p->total_subreads - 1); if (step < (gap << 16)) step = gap << 16; }
		else { step = 6 << 16; if (cr / step > 62) step = cr / 62; }
		if ((1 + cr / step) * gap > 192) {
			svg_set_error("reads of %d bases need %d probes per strand (> 192)", len, (1 + cr / step) * gap);
			return SVG_E_UNSUPPORTED;
		}
	}
	*out = mx;
	return 0;
}

static int launch_unpack(svg_index *h, svg_hostio *io, int slot, uint64_t stride, uint64_t base0, const uint32_t *bases,
                         const uint32_t *xmask, const uint64_t *starts, const uint16_t *lens, uint64_t m, int maxlen,
                         int end, svg_reads *dr, hipStream_t st)
{
	if (slot < 0 || slot > 2) { svg_set_error("chunk slot %d out of range", slot); return SVG_E_ARG; }   // [3]-slot buffers
	// text of end e at [e * m * S, (e + 1) * m * S) of the slot's buffer, offsets likewise
	const uint32_t S = (uint32_t)((maxlen + 3) & ~3);
	size_t need = 2 * m * (size_t)S + 2048, needo = 2 * m * 8 + 64;
	int rc;
	if (end == 0) {
		if ((rc = svg_ensure(h, &io->d_text[slot], &io->d_text_cap[slot], need)) ||
		    (rc = svg_ensure(h, &io->d_offs[slot], &io->d_offs_cap[slot], needo)))
			return rc;
	}
	UnpackParams u;
	u.bases = bases; u.xmask = xmask; u.starts = starts; u.stride = stride; u.base0 = base0; u.lens = lens;
	u.n = (uint32_t)m; u.S = S;
	u.text = (uint32_t *)((uint8_t *)io->d_text[slot] + (size_t)end * m * S);
	u.offs = (uint64_t *)io->d_offs[slot] + (size_t)end * m;
	u.err = h->d_err;
	uint64_t blocks = (m * (S / 4) + 255) / 256, bmax = (uint64_t)h->n_cu * 16;
	if (blocks > bmax) blocks = bmax;
	if (blocks < 1) blocks = 1;
	hipLaunchKernelGGL(unpack_reads, dim3((unsigned)blocks), dim3(256), 0, st, u);
	HIPCHK(hipGetLastError());
	dr->seq = (const char *)u.text;
	dr->offsets = u.offs;
	dr->lens = lens;
	dr->n_reads = m;
	return 0;
}

// the probe kernel reads 2-bit codes straight from the packed reads (align mode)
static void set_packed(VoteJob &job, const svg_packed_reads *pk, int ends, uint64_t b)
{
	job.pp.packed = 1;
	for (int e = 0; e < ends; e++) {
		job.pp.pk_bases[e] = pk[e].bases;
		job.pp.pk_xmask[e] = pk[e].xmask;
		job.pp.pk_starts[e] = pk[e].starts;
		job.pp.pk_stride[e] = pk[e].stride;
		job.pp.pk_base0[e] = b * pk[e].stride;   // sub-batch b.. of a stride-mode stream
	}
}

static int check_packed(const svg_packed_reads *q, const char *who)
{
	if (!q->bases || !q->lens) { svg_set_error("%s: NULL bases/lens", who); return SVG_E_ARG; }
	if (!q->starts && q->stride == 0 && q->n_reads) { svg_set_error("%s: stride 0 without starts", who); return SVG_E_ARG; }
	if (q->n_reads > 0xffffffffull) { svg_set_error("%s: more than 2^32-1 reads in one call", who); return SVG_E_ARG; }
	return 0;
}

extern "C" int svg_vote_batch_device(svg_index *h, const svg_params *p, const svg_reads *r1, const svg_reads *r2,
                                     svg_mapping_result *out, svg_subjunc_result *jout, uint16_t *big_margin, void *stream);

extern "C" int svg_vote_batch_packed_device(svg_index *h, const svg_params *p, const svg_packed_reads *q1,
                                            const svg_packed_reads *q2, svg_mapping_result *out, svg_subjunc_result *jout,
                                            uint16_t *big_margin, void *stream)
{
	if (!h || !p || !q1 || !out) { svg_set_error("svg_vote_batch_packed_device: NULL argument"); return SVG_E_ARG; }
	if (q2 && q2->n_reads != q1->n_reads) { svg_set_error("R1/R2 read counts differ"); return SVG_E_ARG; }
	int rc;
	if ((rc = check_packed(q1, "svg_vote_batch_packed_device")) || (q2 && (rc = check_packed(q2, "svg_vote_batch_packed_device"))))
		return rc;
	if (q1->n_reads == 0) return 0;
	HIPCHK(hipSetDevice(h->device));
	hipStream_t st = stream ? (hipStream_t)stream : h->stream;
	svg_hostio *io;
	if ((rc = io_get(h, &io))) return rc;
	svg_reads dr[2];
	const svg_packed_reads pk[2] = {*q1, q2 ? *q2 : *q1};
	if (p->do_breakpoint_detection || p->do_big_margin_filtering_for_junctions) {
		// subjunc: the wave kernel scores donors on the text, unpacked into the handle's buffer
		if (h->last_pending) HIPCHK(hipStreamWaitEvent(st, h->ev_last, 0));
		const int maxlen = h->max_read_len < SVG_READ_KEEP ? h->max_read_len : SVG_READ_KEEP;
		for (int e = 0; e < (q2 ? 2 : 1); e++)
			if ((rc = launch_unpack(h, io, 0, pk[e].stride, 0, pk[e].bases, pk[e].xmask, pk[e].starts, pk[e].lens, pk[e].n_reads,
			                        maxlen, e, &dr[e], st)))
				return rc;
		return svg_vote_batch_device(h, p, &dr[0], q2 ? &dr[1] : NULL, out, jout, big_margin, st);
	}
	for (int e = 0; e < 2; e++) dr[e] = svg_reads{NULL, NULL, pk[e].lens, pk[e].n_reads};
	return svg_vote_batch_device_packed(h, p, &dr[0], q2 ? &dr[1] : NULL, pk, out, jout, big_margin, st);
}

// ============================================================================ the host pipeline
// Sub-batch i (<= one probe-record chunk) in device slot s = i & 1:
//   up_stream : upload of the reads into d_in[s]
//   stream    : [unpack] + probe + lane kernels             (svg_vote_chunk)
//   stream2   : wave kernel + record compaction + counts    (single-end align: beside the next
//               sub-batch's probe kernel, as in svg_vote_batch_device's chunk pipeline)
//   workers   : expansion of sub-batch i-2 into the caller's buffers
//   down      : download of the compacted records of sub-batch i-2 into staging slot (i-2) % 3
//               (HIP runs these device-to-host copies as blit kernels on the down stream's queue;
//               writing the compact records into mapped host memory from the compaction kernel
//               itself measured slower: 237 vs 318 Mreads/s at C3, the PCIe-bound kernel then
//               sits on the wave kernels' stream)
// Device slots are reused by sub-batch i+2 (i+3) once ev_done (vote + compaction) has fired, compact
// slots by i+3 once ev_down (download) has, a staging slot once its expansion jobs are done.
static int host_pipeline(svg_index *h, const svg_params *p, const svg_reads *a1, const svg_reads *a2,
                         const svg_packed_reads *q1, const svg_packed_reads *q2, svg_mapping_result *out,
                         svg_subjunc_result *jout, uint16_t *big_margin, const char *who)
{
	const bool packed = q1 != NULL;
	const uint64_t n = packed ? q1->n_reads : a1->n_reads;
	const bool pe = packed ? q2 != NULL : a2 != NULL;
	if (pe && (packed ? q2->n_reads : a2->n_reads) != n) { svg_set_error("R1/R2 read counts differ"); return SVG_E_ARG; }
	if (!out) { svg_set_error("%s: NULL out", who); return SVG_E_ARG; }
	if (p->do_breakpoint_detection && !jout) { svg_set_error("do_breakpoint_detection needs jout"); return SVG_E_ARG; }
	if (p->do_big_margin_filtering_for_junctions && !big_margin) { svg_set_error("big-margin filtering needs big_margin"); return SVG_E_ARG; }
	int rc;
	// before anything is sized from multi_best (staging slots, compaction flags: ends * multi_best
	// bits of a uint8 per read)
	if ((rc = svg_check_params(h, p, pe))) return rc;
	if (packed && ((rc = check_packed(q1, who)) || (q2 && (rc = check_packed(q2, who))))) return rc;
	if (!n) return 0;
	const int ends = pe ? 2 : 1, mb = p->multi_best, R = ends * mb;
	const bool jo = p->do_breakpoint_detection != 0, bmo = p->do_big_margin_filtering_for_junctions != 0;
	const bool sjm = jo || bmo;   // subjunc: the wave kernel reads the text (donor scoring)
	HIPCHK(hipSetDevice(h->device));
	// (the copy streams are the handle's: the device's shared stream set, svg_vote.hip)
	svg_hostio *io;
	if ((rc = io_get(h, &io))) return rc;
	{
		const int nt = host_threads();
		if (io->pool && (int)io->pool->th.size() != nt) { delete io->pool; io->pool = NULL; }
		// workers on the GPU's node when this process may run there (else unpinned)
		if (!io->pool) io->pool = new SvgPool(nt, io->node_cpus > 0 ? &io->cpus : NULL);
	}
	uint64_t sub = pe ? (1ull << 19) : (1ull << 20);
	if (svg_get_option("host_sub") > 0) sub = (uint64_t)svg_get_option("host_sub");
	if (sub > n) sub = n;
	const uint16_t *L1 = packed ? q1->lens : a1->lens, *L2 = pe ? (packed ? q2->lens : a2->lens) : NULL;
	const size_t rec_b = (size_t)R * 68, j_b = jo ? (size_t)R * 16 : 0, bm_b = bmo ? (size_t)ends * SVG_BIG_MARGIN_WORDS * 2 : 0;
	const CompLayout CL = comp_layout(sub, R, ends, jo, bmo);
	const size_t o_j = (sub * rec_b + 255) & ~(size_t)255, o_bm = (o_j + sub * j_b + 255) & ~(size_t)255;
	// device slots (probe records, lane lists, full records): 2 -- the probe / lane stream runs one
	// sub-batch ahead of the wave kernel's.  Three slots (two ahead) were measured slower,
	// 114.4-114.9 vs 101.9-102.2 ms/step at C3 (profiles/r04/n/sweep_slots.txt) -- the probe kernel
	// speeds up, the lane and wave kernels slow down more (more kernels on the CUs at once; the
	// probe records, 160 MB per sub-batch, outlive the 256 MB infinity cache)
	const int NS = 2;
	for (int s = 0; s < NS; s++)
		if ((rc = svg_ensure(h, &h->d_out[s], &h->d_out_cap[s], o_bm + sub * bm_b + 64))) return rc;
	for (int s = 0; s < 3; s++) {
		if ((rc = svg_ensure(h, &io->d_comp[s], &io->d_comp_cap[s], CL.bytes))) return rc;
		if ((rc = host_ensure((void **)&io->h_stage[s], &io->h_stage_cap[s], CL.bytes, io->node))) return rc;
	}
	const int saved_len = h->max_read_len;
	// sub-batch boundaries: full sub-batches, ramped at both ends (sub/4, sub/2 first and last) when
	// the batch holds at least 8 of them -- the pipeline fills with a short upload and drains with
	// a short wave kernel + compaction + download + expansion after the last probe kernel; option
	// host_ramp 0 = uniform sub-batches
	std::vector<uint64_t> sb{0};
	{
		// (host_ramp 2: 1/8, 1/4, 1/2 at both ends)
		const int64_t rl = svg_get_option("host_ramp");
		const bool ramp = rl != 0 && n >= 8 * sub && sub >= 64;
		std::vector<uint64_t> steps;   // the ramp's sub-batch sizes, smallest first
		if (ramp) {
			if (rl >= 2) steps.push_back(sub / 8);
			steps.push_back(sub / 4);
			steps.push_back(sub / 2);
		}
		uint64_t tail = 0;
		for (uint64_t x : steps) { sb.push_back(sb.back() + x); tail += x; }
		const uint64_t body_end = n - tail;
		while (sb.back() < body_end) sb.push_back(sb.back() + sub < body_end ? sb.back() + sub : body_end);
		for (size_t k = steps.size(); k-- > 0;) sb.push_back(sb.back() + steps[k]);
	}
	const uint64_t nsub = sb.size() - 1;
	auto sb_b = [&](uint64_t k) { return sb[k]; };
	auto sb_m = [&](uint64_t k) { return sb[k + 1] - sb[k]; };
	hipStream_t st = h->stream;
	if (h->last_pending) HIPCHK(hipStreamWaitEvent(st, h->ev_last, 0));
	for (int k = 0; k < h->nblocks; k++) {
		svg_index *bk = k ? h->blk[k] : h;
		bk->stats_on = h->stats_on;
		if (bk->last_pending && k) HIPCHK(hipStreamWaitEvent(st, bk->ev_last, 0));
		if (h->stats_on) HIPCHK(hipMemsetAsync(bk->d_stats, 0, 32 * sizeof(unsigned long long), st));
	}

	// SVG_PIPE_DEBUG=1: where the host thread waits (seconds per batch)
	const bool dbg = (svg_get_option("debug") & 2) != 0;
	double w_done = 0, w_pool = 0, w_up = 0, w_vote = 0;
	auto now = []() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
	// D2H of the compacted sub-batch j (compact slot j % 3) into staging slot j % 3
	auto download = [&](uint64_t j) -> int {
		const int s3 = (int)(j % 3);
		double t0 = dbg ? now() : 0;
		HIPCHK(hipEventSynchronize(h->ev_done[s3]));
		if (dbg) w_done += now() - t0;
		const uint64_t cnt_rec = io->h_cnt[4 * s3], cnt_j = io->h_cnt[4 * s3 + 1];
		const uint64_t m = sb_m(j);
		const CompLayout C = comp_layout(m, R, ends, jo, bmo);
		t0 = dbg ? now() : 0;
		io->pool->wait(s3);   // staging slot free: expansion of sub-batch j-3 done
		if (dbg) w_pool += now() - t0;
		const uint8_t *src = (const uint8_t *)io->d_comp[s3];
		uint8_t *dst = io->h_stage[s3];
		HIPCHK(hipMemcpyAsync(dst, src, C.o_rec + cnt_rec * 68, hipMemcpyDeviceToHost, h->down_stream));
		if (jo) HIPCHK(hipMemcpyAsync(dst + C.o_jflags, src + C.o_jflags, C.o_jrec - C.o_jflags + cnt_j * 16,
		                              hipMemcpyDeviceToHost, h->down_stream));
		if (bmo) HIPCHK(hipMemcpyAsync(dst + C.o_bm, src + C.o_bm, m * bm_b, hipMemcpyDeviceToHost, h->down_stream));
		HIPCHK(hipEventRecord(h->ev_down[s3], h->down_stream));
		return 0;
	};
	// expansion of sub-batch k (staging slot k % 3) into the caller's buffers
	auto expand = [&](uint64_t k) -> int {
		const int s3 = (int)(k % 3);
		HIPCHK(hipEventSynchronize(h->ev_down[s3]));
		const uint64_t b = sb_b(k), m = sb_m(k);
		const CompLayout C = comp_layout(m, R, ends, jo, bmo);
		const uint8_t *stg = io->h_stage[s3];
		const uint32_t tiles = C.tiles, per_job = 128;   // 8192 reads per job
		for (uint32_t t0 = 0; t0 < tiles; t0 += per_job) {
			const uint32_t t1 = t0 + per_job < tiles ? t0 + per_job : tiles;
			io->pool->post(s3, [=]() {
				// a tile's records are assembled in a cache-resident buffer and leave with streaming
				// stores: the caller's array is written once and never read, so plain stores would
				// also read every line first (read-for-ownership) -- twice the host memory traffic
				alignas(64) uint8_t tbuf[64 * 6 * 68];
				const uint8_t *flags = stg + C.o_flags;
				const uint32_t *tb = (const uint32_t *)(stg + C.o_tile);
				for (uint32_t t = t0; t < t1; t++) {
					const uint64_t r0 = (uint64_t)t * 64, r1 = r0 + 64 < m ? r0 + 64 : m;
					const uint8_t *rec = stg + C.o_rec + (size_t)tb[t] * 68;
					uint8_t *const od = (uint8_t *)out + (b + r0) * rec_b;
					const size_t tbytes = (size_t)(r1 - r0) * rec_b;
					const bool nt = tbytes <= sizeof tbuf && (((uintptr_t)od | tbytes) & 15) == 0;
					uint8_t *o = nt ? tbuf : od;
					for (uint64_t r = r0; r < r1; r++) {
						const uint32_t f = flags[r];
						for (int q = 0; q < R; q++, o += 68)
							if ((f >> q) & 1u) { memcpy(o, rec, 68); rec += 68; }
							else memset(o, 0, 68);
					}
					if (nt) stream_out(od, tbuf, tbytes);
					if (jo) {
						const uint8_t *jf = stg + C.o_jflags;
						const uint32_t *jt = (const uint32_t *)(stg + C.o_jtile);
						const uint8_t *jr = stg + C.o_jrec + (size_t)jt[t] * 16;
						uint8_t *const jdd = (uint8_t *)jout + (b + r0) * j_b;
						const size_t jbytes = (size_t)(r1 - r0) * j_b;
						const bool jnt = jbytes <= sizeof tbuf && (((uintptr_t)jdd | jbytes) & 15) == 0;
						uint8_t *jd = jnt ? tbuf : jdd;
						for (uint64_t r = r0; r < r1; r++) {
							const uint32_t f = jf[r];
							for (int q = 0; q < R; q++, jd += 16)
								if ((f >> q) & 1u) { memcpy(jd, jr, 16); jr += 16; }
								else memset(jd, 0, 16);
						}
						if (jnt) stream_out(jdd, tbuf, jbytes);
					}
					if (bmo) memcpy((uint8_t *)big_margin + (b + r0) * bm_b, stg + C.o_bm + r0 * bm_b, (r1 - r0) * bm_b);
				}
				_mm_sfence();   // streaming stores visible before the job counts as done
			});
		}
		return 0;
	};

	// upload of sub-batch u into input slot u % 3 (run one sub-batch ahead of the vote, so the
	// copy is in flight while the GPU still works on the previous sub-batches)
	struct Up {
		size_t o_seq[2], o_off[2], o_len[2], o_bases[2], o_x[2], o_st[2];
		uint64_t lo[2], wlo[2], xlo[2];
		int maxlen;
	} up[3];
	auto upload = [&](uint64_t u) -> int {
		const int s3 = (int)(u % 3);
		const uint64_t b = sb_b(u), m = sb_m(u);
		Up &U = up[s3];
		memset(&U, 0, sizeof U);
		int rc2;
		if ((rc2 = sub_max_len(h, p, L1, L2, b, m, &U.maxlen))) return rc2;
		// slot u % 3 was last read by sub-batch u-3 (its lengths, until its wave kernel is done)
		if (u >= 3) HIPCHK(hipStreamWaitEvent(h->up_stream, h->ev_done[u % 3], 0));
		size_t in_bytes = 0;
		struct Part { const void *src; size_t off, bytes; } parts[8];
		int np_ = 0;
		auto add = [&](const void *src, size_t bytes) {
			parts[np_].src = src; parts[np_].off = in_bytes; parts[np_].bytes = bytes; np_++;
			in_bytes = (in_bytes + bytes + 255) & ~(size_t)255;
			return parts[np_ - 1].off;
		};
		for (int e = 0; e < ends; e++) {
			if (!packed) {
				const svg_reads *rr = e ? a2 : a1;
				uint64_t mn = ~0ull, mx = 0;
				for (uint64_t r = b; r < b + m; r++) {
					if (rr->offsets[r] < mn) mn = rr->offsets[r];
					if (rr->offsets[r] + rr->lens[r] > mx) mx = rr->offsets[r] + rr->lens[r];
				}
				U.lo[e] = mn;
				U.o_seq[e] = add(rr->seq + mn, mx - mn);
				U.o_off[e] = add(rr->offsets + b, 8 * m);
				U.o_len[e] = add(rr->lens + b, 2 * m);
			} else {
				const svg_packed_reads *q = e ? q2 : q1;
				uint64_t mn = ~0ull, mx = 0;
				if (q->starts) {
					for (uint64_t r = b; r < b + m; r++) {
						if (q->starts[r] < mn) mn = q->starts[r];
						if (q->starts[r] + q->lens[r] > mx) mx = q->starts[r] + q->lens[r];
					}
				} else {
					// read r in bases [r * stride, r * stride + min(lens[r], stride))
					mn = b * q->stride;
					mx = (b + m) * q->stride;
				}
				if (mx < mn) mx = mn;
				U.wlo[e] = mn >> 4;
				U.o_bases[e] = add(q->bases + U.wlo[e], 4 * (((mx + 15) >> 4) - U.wlo[e]));
				if (q->xmask) { U.xlo[e] = mn >> 5; U.o_x[e] = add(q->xmask + U.xlo[e], 4 * (((mx + 31) >> 5) - U.xlo[e])); }
				if (q->starts) U.o_st[e] = add(q->starts + b, 8 * m);
				U.o_len[e] = add(q->lens + b, 2 * m);
			}
		}
		if ((rc2 = svg_ensure(h, &h->d_in[s3], &h->d_in_cap[s3], in_bytes + 64))) return rc2;
		uint8_t *din = (uint8_t *)h->d_in[s3];
		for (int k = 0; k < np_; k++)
			if (parts[k].bytes) HIPCHK(hipMemcpyAsync(din + parts[k].off, parts[k].src, parts[k].bytes, hipMemcpyHostToDevice, h->up_stream));
		HIPCHK(hipEventRecord(h->ev_up[s3], h->up_stream));
		return 0;
	};

	bool overlap_any = false;
	rc = upload(0);
	// iteration i: upload i+1, vote i, download i-2, expand i-3 -- the host blocks on sub-batch
	// i-2 only, with i-1 and i already queued behind it on the GPU
	for (uint64_t i = 0; i < nsub + 3 && !rc; i++) {
		if (i >= nsub) goto tail;
		{
		const int s = (int)(i % (uint64_t)NS), s3 = (int)(i % 3);
		const uint64_t b = sb_b(i), m = sb_m(i);
		double tu = dbg ? now() : 0;
		if (i + 1 < nsub && (rc = upload(i + 1))) break;
		if (dbg) { w_up += now() - tu; tu = now(); }
		uint8_t *dout;
		hipStream_t st2 = st;
		{
		const Up &U = up[s3];
		uint8_t *din = (uint8_t *)h->d_in[s3];
		// ---- vote on stream (probe, lane) / stream2 (wave); slot s free once sub-batch i-2 is done
		HIPCHK(hipStreamWaitEvent(st, h->ev_up[s3], 0));
		if (i >= (uint64_t)NS) HIPCHK(hipStreamWaitEvent(st, h->ev_done[(i - NS) % 3], 0));
		h->max_read_len = U.maxlen;
		svg_reads dr[2];
		svg_packed_reads pk[2];
		for (int e = 0; e < ends && !rc; e++) {
			if (!packed) {
				// the caller's offsets go up unchanged: the device text pointer is rebased instead
				dr[e].seq = (const char *)(din + U.o_seq[e]) - U.lo[e];
				dr[e].offsets = (const uint64_t *)(din + U.o_off[e]);
				dr[e].lens = (const uint16_t *)(din + U.o_len[e]);
				dr[e].n_reads = m;
			} else {
				// the uploaded word ranges keep the stream's base numbering: the device pointers
				// are rebased by the first uploaded word (starts and b * stride stay global)
				const svg_packed_reads *q = e ? q2 : q1;
				pk[e].bases = (const uint32_t *)(din + U.o_bases[e]) - U.wlo[e];
				pk[e].xmask = q->xmask ? (const uint32_t *)(din + U.o_x[e]) - U.xlo[e] : NULL;
				pk[e].starts = q->starts ? (const uint64_t *)(din + U.o_st[e]) : NULL;
				pk[e].stride = q->stride;
				pk[e].lens = (const uint16_t *)(din + U.o_len[e]);
				pk[e].n_reads = m;
				if (sjm) rc = launch_unpack(h, io, s, q->stride, b * q->stride, pk[e].bases, pk[e].xmask, pk[e].starts, pk[e].lens, m,
				                            U.maxlen, e, &dr[e], st);
				else dr[e] = svg_reads{NULL, NULL, pk[e].lens, m};   // the probe kernel reads the 2-bit codes
			}
		}
		if (rc) break;
		dout = (uint8_t *)h->d_out[s];
		VoteJob job;
		if ((rc = svg_vote_prepare(h, p, &dr[0], pe ? &dr[1] : NULL, (svg_mapping_result *)dout,
		                           jo ? (svg_subjunc_result *)(dout + o_j) : NULL, bmo ? (uint16_t *)(dout + o_bm) : NULL, &job)))
			break;
		if (packed && !sjm) set_packed(job, pk, ends, b);
		// a multi-block index votes its blocks in order on one stream (each later block merges with
		// the records the earlier ones left)
		const bool overlap = job.overlap_mode && nsub > 1 && m <= job.chunk && h->nblocks < 2;
		overlap_any = overlap_any || overlap;
		st2 = overlap ? h->stream2 : st;
		for (uint64_t c0 = 0; c0 < m && !rc; c0 += job.chunk)   // one chunk unless reads are long
			rc = svg_vote_chunk(h, &job, c0, m - c0 < job.chunk ? m - c0 : job.chunk, s, st, st2);
		for (int k = 1; k < h->nblocks && !rc; k++) {
			svg_index *bk = h->blk[k];
			bk->max_read_len = U.maxlen;
			VoteJob jk;
			if ((rc = svg_vote_prepare(bk, p, &dr[0], pe ? &dr[1] : NULL, (svg_mapping_result *)dout,
			                           jo ? (svg_subjunc_result *)(dout + o_j) : NULL, bmo ? (uint16_t *)(dout + o_bm) : NULL, &jk)))
				break;
			if (packed && !sjm) set_packed(jk, pk, ends, b);
			for (uint64_t c0 = 0; c0 < m && !rc; c0 += jk.chunk)
				rc = svg_vote_chunk(bk, &jk, c0, m - c0 < jk.chunk ? m - c0 : jk.chunk, 0, st, st);
		}
		if (rc) break;
		if (dbg) w_vote += now() - tu;
		}
		// ---- compaction into compact slot s3 (free once sub-batch i-3's download is done)
		if (i >= 3) HIPCHK(hipStreamWaitEvent(st2, h->ev_down[s3], 0));
		{
			const CompLayout C = comp_layout(m, R, ends, jo, bmo);
			uint8_t *dc = (uint8_t *)io->d_comp[s3];
			HIPCHK(hipMemsetAsync(io->d_cnt + 4 * s3, 0, 16, st2));
			hipLaunchKernelGGL(compact_records<17>, dim3(C.tiles), dim3(64), 2 * 64 * R * 17 * 4, st2, (const uint32_t *)dout, R,
			                   (uint32_t)m, (uint32_t *)(dc + C.o_rec), dc + C.o_flags, (uint32_t *)(dc + C.o_tile), io->d_cnt + 4 * s3);
			HIPCHK(hipGetLastError());
			if (jo) {
				hipLaunchKernelGGL(compact_records<4>, dim3(C.tiles), dim3(64), 2 * 64 * R * 4 * 4, st2, (const uint32_t *)(dout + o_j),
				                   R, (uint32_t)m, (uint32_t *)(dc + C.o_jrec), dc + C.o_jflags, (uint32_t *)(dc + C.o_jtile),
				                   io->d_cnt + 4 * s3 + 1);
				HIPCHK(hipGetLastError());
			}
			if (bmo) HIPCHK(hipMemcpyAsync(dc + C.o_bm, dout + o_bm, m * bm_b, hipMemcpyDeviceToDevice, st2));
			HIPCHK(hipMemcpyAsync(io->h_cnt + 4 * s3, io->d_cnt + 4 * s3, 16, hipMemcpyDeviceToHost, st2));
			HIPCHK(hipEventRecord(h->ev_done[s3], st2));
		}
		}
	tail:
		// ---- sub-batch i-2 goes down, i-3 is expanded
		if (i >= 2 && i - 2 < nsub && (rc = download(i - 2))) break;
		if (i >= 3 && i - 3 < nsub && (rc = expand(i - 3))) break;
	}
	{
		const double t0 = dbg ? now() : 0;
		for (int s = 0; s < 3; s++) io->pool->wait(s);
		if (dbg)
			fprintf(stderr, "[svg] %s: %llu sub-batches of %llu; host spent %.1f ms issuing uploads, %.1f ms issuing "
			        "votes, waited %.1f ms on vote+compaction, %.1f ms on expansion, %.1f ms on the final expansion\n",
			        who, (unsigned long long)nsub, (unsigned long long)sub, w_up * 1e3, w_vote * 1e3, w_done * 1e3,
			        w_pool * 1e3, (now() - t0) * 1e3);
	}
	h->max_read_len = saved_len;
	// join the second stream; later calls on the handle start after all of this
	for (int s = 0; s < 3 && overlap_any && !rc; s++) HIPCHK(hipStreamWaitEvent(st, h->ev_done[s], 0));
	if (!rc) {
		HIPCHK(hipEventRecord(h->ev_last, st));
		h->last_pending = 1;
	}
	hipError_t e1 = hipStreamSynchronize(st), e2 = hipStreamSynchronize(h->stream2),
	           e3 = hipStreamSynchronize(h->up_stream), e4 = hipStreamSynchronize(h->down_stream);
	if (rc) return rc;
	if (e1 != hipSuccess || e2 != hipSuccess || e3 != hipSuccess || e4 != hipSuccess) {
		hipError_t e = e1 != hipSuccess ? e1 : e2 != hipSuccess ? e2 : e3 != hipSuccess ? e3 : e4;
		svg_set_error("HIP error %s in %s", hipGetErrorString(e), who);
		return SVG_E_DEVICE;
	}
	if (h->stats_on) {
		svg_batch_stats acc = {};
		for (int k = 0; k < h->nblocks; k++) {
			unsigned long long sv[5];
			HIPCHK(hipMemcpy(sv, (k ? h->blk[k] : h)->d_stats, sizeof sv, hipMemcpyDeviceToHost));
			acc.probes += sv[0];
			acc.bucket_items += sv[1];
			acc.hits += sv[2];
			acc.results = sv[3];   // the last block's records are the final ones
			acc.deferred += sv[4];
		}
		h->last_stats = acc;
	}
	return svg_device_status(h);
}

// ============================================================================ entry points
extern "C" int svg_vote_batch(svg_index *h, const svg_params *p, const svg_reads *r1, const svg_reads *r2,
                              svg_mapping_result *out, svg_subjunc_result *jout, uint16_t *big_margin)
{
	if (!h || !p || !r1) { svg_set_error("svg_vote_batch: NULL argument"); return SVG_E_ARG; }
	return host_pipeline(h, p, r1, r2, NULL, NULL, out, jout, big_margin, "svg_vote_batch");
}

extern "C" int svg_vote_batch_packed(svg_index *h, const svg_params *p, const svg_packed_reads *q1,
                                     const svg_packed_reads *q2, svg_mapping_result *out, svg_subjunc_result *jout,
                                     uint16_t *big_margin)
{
	if (!h || !p || !q1) { svg_set_error("svg_vote_batch_packed: NULL argument"); return SVG_E_ARG; }
	return host_pipeline(h, p, NULL, NULL, q1, q2, out, jout, big_margin, "svg_vote_batch_packed");
}

// ============================================================================ host packer
// code | exception << 2 per character
static uint8_t g_pack_lut[256];
static std::once_flag g_pack_once;

extern "C" int64_t svg_pack_reads(const svg_reads *in, uint64_t stride, uint32_t *bases, uint32_t *xmask, uint64_t *starts,
                                  int threads)
{
	if (!in || !bases || !xmask) { svg_set_error("svg_pack_reads: NULL argument"); return SVG_E_ARG; }
	std::call_once(g_pack_once, [] {
		for (int c = 0; c < 256; c++) g_pack_lut[c] = (uint8_t)(pack_code((unsigned char)c) | (pack_exception((unsigned char)c) ? 4u : 0u));
	});
	const uint64_t n = in->n_reads;
	uint64_t total = 0;
	if (starts) {
		for (uint64_t i = 0; i < n; i++) { starts[i] = total; total += in->lens[i]; }
	} else {
		if (n && stride == 0) { svg_set_error("svg_pack_reads: stride 0 without starts"); return SVG_E_ARG; }
		for (uint64_t i = 0; i < n; i++)
			if (in->lens[i] > stride) { svg_set_error("svg_pack_reads: read %llu longer than the stride", (unsigned long long)i); return SVG_E_ARG; }
		total = n * stride;
	}
	const uint64_t groups = (total + 31) / 32;   // 32 bases: two base words, one mask word
	if (threads < 1) threads = 1;
	if ((uint64_t)threads > groups / 4096 + 1) threads = (int)(groups / 4096 + 1);
	std::vector<int64_t> exc((size_t)threads, 0);
	auto work = [&](int t) {
		const uint64_t g0 = groups * t / threads, g1 = groups * (t + 1) / threads;
		if (g0 >= g1) return;
		// the read holding base 32 * g0
		uint64_t k = 32 * g0, r;
		if (starts) {
			uint64_t lo = 0, hi = n;   // last read with starts[r] <= k
			while (hi - lo > 1) { const uint64_t mid = (lo + hi) / 2; if (starts[mid] <= k) lo = mid; else hi = mid; }
			r = lo;
		} else r = k / stride;
		int64_t ne = 0;
		for (uint64_t g = g0; g < g1; g++) {
			uint32_t w[2] = {0, 0}, xm = 0;
			for (int j = 0; j < 32; j++, k++) {
				if (k >= total) break;
				uint64_t rs, re;
				for (;;) {
					rs = starts ? starts[r] : r * stride;
					re = rs + in->lens[r];
					if (k < (starts ? re : rs + stride) || r + 1 >= n) break;
					r++;
				}
				if (k < rs || k >= re) continue;   // stride padding: code 0, no exception
				const uint8_t v = g_pack_lut[(unsigned char)in->seq[in->offsets[r] + (k - rs)]];
				w[j >> 4] |= (uint32_t)(v & 3u) << (30 - 2 * (j & 15));
				if (v & 4u) { xm |= 1u << (31 - j); ne++; }
			}
			bases[2 * g] = w[0];
			if (2 * g + 1 < (total + 15) / 16) bases[2 * g + 1] = w[1];
			xmask[g] = xm;
		}
		exc[(size_t)t] = ne;
	};
	std::vector<std::thread> th;
	for (int t = 1; t < threads; t++) th.emplace_back(work, t);
	work(0);
	for (auto &x : th) x.join();
	int64_t ne = 0;
	for (auto v : exc) ne += v;
	return ne;
}
