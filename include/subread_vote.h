/*
 * subread_vote.h -- C ABI of the MI355X seed-and-vote read-alignment hot path.
 *
 * Drop-in boundary for the voting step of Subread v2.0.6 (subread-align /
 * subjunc).  In the reference the step is the internal function
 *     int do_voting(global_context_t*, thread_context_t*)        core.c:3049
 * run once per pthread by run_in_thread(STEP_VOTING)             core.c:3366
 * It pulls reads from fetch_next_read_pair (core.c:1121), probes the sorted
 * hash table with gehash_go_X (sorted-hashtable.c:937), selects the top-K
 * candidates with process_voting_junction_PE_topK (core-junction.c:2199) and
 * writes up to multi_best mapping_result_t per read end into the bigtable
 * (core-bigtable.c:127) -- plus subjunc_result_t and the big-margin records in
 * subjunc mode.  svg_vote_batch() replaces that whole step for a batch of reads:
 * reads (ASCII, exactly what fetch_next_read_pair hands to do_voting before the
 * -S reversal) go in, the same bigtable records come out, byte for byte.
 *
 * Conventions (mirroring the reference): functions return 0 on success and a
 * negative SVG_E_* code on failure; the text of the last error of the calling
 * thread is available from svg_last_error().  The caller owns every host
 * buffer; the library owns device memory and streams.  One handle per GPU;
 * calls on one handle are serialised by the caller (one host thread).
 *
 * Nothing in this header depends on HIP or torch types.
 */
#ifndef SUBREAD_VOTE_H
#define SUBREAD_VOTE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SVG_ABI_VERSION 2

/* reference constants (subread.h:73,88,216-217; core-junction.c:3569) */
#define SVG_MAX_READ_LENGTH       1210   /* MAX_READ_LENGTH == index padding */
/* the reference's reader keeps at most MAX_READ_LENGTH-1 bases of a read line
 * (read_line, input-files.c:277); longer reads are truncated the same way here */
#define SVG_READ_KEEP             (SVG_MAX_READ_LENGTH - 1)
#define SVG_MAX_INDEL_SECTIONS    7
#define SVG_VOTE_TABLE_SIZE       30     /* GENE_VOTE_TABLE_SIZE */
#define SVG_VOTE_SPACE            24     /* GENE_VOTE_SPACE */
#define SVG_BIG_MARGIN_WORDS      9      /* config.big_margin_record_size */
#define SVG_NEGATIVE_STRAND_FLAG  8      /* CORE_IS_NEGATIVE_STRAND in result_flags */

/* error codes */
#define SVG_OK               0
#define SVG_E_ARG          (-1)   /* bad argument / NULL pointer */
#define SVG_E_IO           (-2)   /* index file missing / unreadable */
#define SVG_E_FORMAT       (-3)   /* index file malformed */
#define SVG_E_UNSUPPORTED  (-4)   /* configuration outside the drop-in contract */
#define SVG_E_DEVICE       (-5)   /* HIP runtime failure */
#define SVG_E_NOMEM        (-6)

/* mapping_result_t, core.h:350-370 -- identical layout (68 bytes). */
typedef struct svg_mapping_result {
	uint32_t selected_position;
	int16_t  result_flags;
	int16_t  read_length;
	int16_t  selected_votes;
	int16_t  used_subreads_in_vote;
	uint8_t  noninformative_subreads_in_vote;
	int8_t   indels_in_confident_coverage;
	int8_t   is_fully_covered;
	uint8_t  _pad0;
	int16_t  selected_indel_record[SVG_MAX_INDEL_SECTIONS * 3 + 1];
	uint16_t confident_coverage_start;
	uint16_t confident_coverage_end;
	int16_t  subread_quality;
	uint16_t _pad1;
} svg_mapping_result;

/* subjunc_result_t, core.h:397-410 -- identical layout (16 bytes). */
typedef struct svg_subjunc_result {
	int16_t  split_point;
	int16_t  minor_votes;
	int8_t   double_indel_offset;
	int8_t   indel_at_junction;
	int8_t   small_side_increasing_coordinate;
	int8_t   large_side_increasing_coordinate;
	uint32_t minor_position;
	uint16_t minor_coverage_start;
	uint16_t minor_coverage_end;
} svg_subjunc_result;

/*
 * Voting parameters: the subset of configuration_t (core.h:128-253) the vote
 * path reads.  svg_params_default() fills them exactly as the reference does:
 * init_global_context (core-indel.c:4399-4538), then parse_opts_aligner /
 * parse_opts_subjunc (core-interface-aligner.c:256, core-interface-subjunc.c:255),
 * then the runtime overrides of load_global_context (core.c:4075-4094).
 */
typedef struct svg_params {
	int32_t total_subreads;               /* -n                      (10 align, 14 subjunc) */
	int32_t min_votes_first;              /* -m minimum_subread_for_first_read  (3 / 1)   */
	int32_t min_votes_second;             /* -p minimum_subread_for_second_read (1)       */
	int32_t max_indel_length;             /* -I  (voting uses min(16, I))        (5)      */
	int32_t multi_best;                   /* multi_best_reads                    (3)      */
	int32_t top_scores;                   /*                                     (3)      */
	int32_t max_vote_simples;             /* 3 SE / 64 PE, max'ed with -B                 */
	int32_t max_vote_combinations;        /* 3, max'ed with -B                            */
	int32_t max_vote_number_cutoff;       /*                                     (2)      */
	int32_t min_pair_distance;            /* -d                                  (50)     */
	int32_t max_pair_distance;            /* -D                                  (600)    */
	int32_t reverse_r1;                   /* is_first_read_reversed  (-S)        (0)      */
	int32_t reverse_r2;                   /* is_second_read_reversed (-S)        (1)      */
	int32_t do_breakpoint_detection;      /* subjunc                             (0 / 1)  */
	int32_t do_big_margin_filtering_for_junctions; /* subjunc                    (0 / 1)  */
	int32_t big_margin_record_size;       /*                                     (9)      */
	int32_t maximum_intron_length;        /*                                     (500000) */
	int32_t prefer_donor_receptor_junctions; /*                                  (1)      */
	int32_t check_donor_at_junctions;     /*                                     (1)      */
	int32_t max_insertion_at_junctions;   /*                                     (0)      */
	int32_t more_accurate_fusions;        /*                                     (1)      */
} svg_params;

#define SVG_PROGRAM_ALIGN   0   /* subread-align */
#define SVG_PROGRAM_SUBJUNC 1   /* subjunc */
void svg_params_default(svg_params *p, int program, int paired_end);

/*
 * A batch of reads as ASCII text.  Read i is seq[offsets[i] .. offsets[i]+lens[i]).
 * Reads are given as the FASTQ holds them (after trimming); the -S reversal
 * (reverse_r1 / reverse_r2) is applied inside the library exactly like
 * fetch_next_read_pair (core.c:1186-1198).  For paired-end input r1 and r2 hold
 * the same number of reads.  Read numbering in a batch = array order.
 */
typedef struct svg_reads {
	const char     *seq;
	const uint64_t *offsets;
	const uint16_t *lens;
	uint64_t        n_reads;
} svg_reads;

/*
 * The same reads 2-bit packed: ~4x fewer bytes to move than ASCII.
 *   bases : base2int codes (subread.h:238: A=0 G=1 C=2 T=3; any other character 2 if it
 *           sorts below 'G', else 3), 16 per word; base k of the stream in bits
 *           31-2(k%16) .. 30-2(k%16) of word k/16, so 16 bases starting at a word boundary
 *           read as genekey2int's key (input-files.c:1232).
 *   xmask : NULL when every base is A/C/G/T/U; else 1 bit per base (bit 31-(k%32) of word
 *           k/32) set for any other character (N, '.', lowercase, IUPAC ...).  Those all
 *           complement to 'N' in reverse_read (input-files.c:1111) and never match the
 *           genome there; 'U' behaves as 'T' everywhere and packs as T.  (A read holds no
 *           NUL byte -- it would end the reference's C string.)
 *   starts: base index of read i in the stream; NULL = i * stride.
 * Read i = bases starts[i] .. starts[i]+lens[i]-1.  svg_pack_reads() builds this form.
 */
typedef struct svg_packed_reads {
	const uint32_t *bases;
	const uint32_t *xmask;
	const uint64_t *starts;
	uint64_t        stride;
	const uint16_t *lens;
	uint64_t        n_reads;
} svg_packed_reads;

/* Pack ASCII reads: with starts != NULL the reads go back to back (starts[i] filled in,
 * bases sized ceil(sum(lens)/16) words, xmask ceil(sum(lens)/32)); with starts == NULL read
 * i goes to base i*stride (every lens[i] <= stride; n*stride bases).  Returns the number of
 * exception bases (0: the caller may pass xmask = NULL to the vote) or a negative SVG_E_*. */
int64_t svg_pack_reads(const svg_reads *in, uint64_t stride, uint32_t *bases, uint32_t *xmask, uint64_t *starts,
                       int threads);

/* opaque index handle: owns the HBM copy of every <prefix>.NN.b.tab / .array block and .reads */
typedef struct svg_index svg_index;

typedef struct svg_index_info {
	uint64_t items;              /* hashed 16-mers in the .tab                 */
	uint32_t buckets;            /* buckets_number                             */
	int32_t  index_gap;          /* 1 (-F full index) or 3 (gapped)            */
	int32_t  padding;            /* 1210                                       */
	uint32_t array_length;       /* .array length (bases incl. padding)        */
	uint32_t n_chromosomes;
	uint64_t device_bytes;       /* HBM held by the handle                     */
	int32_t  device;             /* HIP device ordinal                         */
	uint32_t array_values_bytes; /* bytes of the packed .array image           */
	int32_t  n_blocks;           /* index blocks (<prefix>.NN.b.*); the fields above
	                                but device_bytes describe block 00           */
} svg_index_info;

/* Load a base-space index as written by subread-buildindex -- "<prefix>.NN.b.tab" and
 * "<prefix>.NN.b.array" for every block NN = 00, 01, ... and "<prefix>.reads" -- into HBM of
 * `device`.  All blocks stay resident; a vote runs them in order, each later block merging
 * with the records the earlier ones left (read_chunk_circles, core.c:3567-3613), so a
 * multi-block index gives the reference's records for the same reads. */
int  svg_index_open(const char *prefix, int device, svg_index **out);
/* The same for n devices at once (out[k] on devices[k]; a device may repeat: several replicas on
 * one GPU): the files are read, walked and staged once and every staged run is copied to every
 * replica -- an 8-GPU node loads the index once instead of eight times.  All or nothing: on an
 * error no handle is left open. */
int  svg_index_open_devices(const char *prefix, const int *devices, int n, svg_index **out);
void svg_index_close(svg_index *idx);
int  svg_index_get_info(const svg_index *idx, svg_index_info *out);

/*
 * Build a single-block index straight into HBM (same bytes as svg_build_index /
 * subread-buildindex), from a FASTA file or from in-memory contigs; when
 * save_prefix is not NULL the reference-format files are also written there.
 */
int  svg_index_build(const char *fasta, int gap, int memory_mb, int force_one_block,
                     int repeat_threshold, int device, const char *save_prefix, svg_index **out);
int  svg_index_build_mem(const char *const *names, const char *const *seqs, const uint64_t *lens,
                         uint32_t n_contigs, int gap, int memory_mb, int force_one_block,
                         int repeat_threshold, int device, const char *save_prefix, svg_index **out);
/* Copy block 00 of the index back to host arrays (any pointer may be NULL): bstart[buckets+1],
 * keys[items], vals[items], values[array_values_bytes], chr_end[n_chromosomes]. */
int  svg_index_export(const svg_index *idx, uint32_t *bstart, int16_t *keys, uint32_t *vals,
                      uint8_t *values, uint32_t *chr_end);

/*
 * Vote a batch.  Host buffers in, host buffers out (synchronous).
 *   out   : n_reads * ends * multi_best records, index ((read*ends)+end)*multi_best+best
 *   jout  : same shape, subjunc_result_t; required iff do_breakpoint_detection
 *   big_margin : n_reads * ends * SVG_BIG_MARGIN_WORDS; required iff
 *           do_big_margin_filtering_for_junctions (reference bigtable
 *           big_margin_data, core.h:453)
 * r2 == NULL means single-end.  Output buffers are fully overwritten (the
 * reference zeroes the bigtable per chunk, core-bigtable.c:84-125).
 */
int svg_vote_batch(svg_index *idx, const svg_params *p,
                   const svg_reads *r1, const svg_reads *r2,
                   svg_mapping_result *out, svg_subjunc_result *jout,
                   uint16_t *big_margin);
/* The same from 2-bit packed reads (host buffers).  Both host entry points run a sub-batch
 * pipeline: upload of sub-batch i+1, vote of i (probe + lane kernels) beside the wave kernel and
 * compaction of i-1, download of i-2 (only the non-zero records, compacted on the GPU) and
 * expansion of i-3 into `out` by worker threads overlap.  Workers: svg_host_threads().  Pinned caller buffers copy fastest. */
int svg_vote_batch_packed(svg_index *idx, const svg_params *p,
                          const svg_packed_reads *r1, const svg_packed_reads *r2,
                          svg_mapping_result *out, svg_subjunc_result *jout,
                          uint16_t *big_margin);

/*
 * Same computation on device-resident buffers, asynchronous on `hip_stream`
 * (a hipStream_t passed as void*, NULL = the handle's own stream).  Every
 * pointer in r1/r2 and the outputs is a device pointer.
 */
int svg_vote_batch_device(svg_index *idx, const svg_params *p,
                          const svg_reads *r1, const svg_reads *r2,
                          svg_mapping_result *out, svg_subjunc_result *jout,
                          uint16_t *big_margin, void *hip_stream);
/* Packed reads in device memory (unpacked on the GPU into a buffer of the handle, sized by
 * svg_set_max_read_length's bound), asynchronous on `hip_stream`. */
int svg_vote_batch_packed_device(svg_index *idx, const svg_params *p,
                                 const svg_packed_reads *r1, const svg_packed_reads *r2,
                                 svg_mapping_result *out, svg_subjunc_result *jout,
                                 uint16_t *big_margin, void *hip_stream);

/*
 * Equal-key runs of arbitrary subread keys in one index block: cellCounts' hit-list lookup
 * (prefill_votes, cell-counts.c:432-491) on the GPU.  For key i: bucket b = key % buckets,
 * binary search of (short)(key / buckets) in the bucket's keys, then prefill_votes' step-down
 * widening, exactly.  first[i] = bucket-local index of the run's first item (the reference's
 * start_location_in_index = bucket->item_values + first[i]), count[i] = run length (its
 * votes[i]; 0 = absent, first[i] = 0).  svg_probe_keys takes host buffers (synchronous);
 * svg_probe_keys_device device buffers, asynchronous on hip_stream (NULL: the handle's).
 */
int svg_probe_keys(svg_index *idx, int block, const uint32_t *keys, uint64_t n,
                   uint32_t *first, uint32_t *count);
int svg_probe_keys_device(svg_index *idx, int block, const uint32_t *keys, uint64_t n,
                          uint32_t *first, uint32_t *count, void *hip_stream);

/*
 * Fragile junction voting of subjunc reads longer than 160 bases (core_fragile_junction_voting,
 * core-junction.c:5151-5422; do_voting runs it for every index block, strand and read end,
 * core.c:3138-3142).  The read (strand 0: as fetched after the -S reversal, strand 1: its
 * reverse_read) is cut into ~60-base windows; each window is voted with gehash_go_q
 * (sorted-hashtable.c:515-933: every item of the key's equal-key run from the first one, the
 * go_X tally without shift-indel rounds, tolerance 5) over subreads every 3.00001 bases, then:
 *   - every slot with the top vote count whose indel recorder has a second section is reported
 *     (svg_fragile_slot) -- the reference aligns those on the host (core_dynamic_align) into
 *     indel events;
 *   - select_best_vote + core_select_best_matching_halves pick a second half, and
 *     core13_test_donor (GT..AG / CT..AC donors, 17-base match windows) decides whether the
 *     window supports a junction (small_side, large_side, is_GTAG).
 * svg_fragile_batch runs all of it on the GPU for a batch (host buffers, synchronous; reads as
 * svg_vote_batch takes them, p must be subjunc parameters); the result arrays are owned by the
 * library until svg_fragile_free.  The events are made on the host by svg_events_add_batch2
 * (include/subread_events.h), in the reference's order.
 */
typedef struct svg_fragile_window {
	uint32_t read;             /* read (pair) number in the batch */
	uint8_t  block;            /* index block */
	uint8_t  strand;           /* 0: the read as fetched, 1: reverse_read of it */
	uint8_t  end;              /* 0: R1, 1: R2 */
	uint8_t  window;           /* window number */
	uint16_t start, length;    /* window_cursor and read_len of the window */
	uint8_t  junction;         /* 1: core13_test_donor accepted a split point */
	uint8_t  gtag;             /* its is_GTAG */
	uint16_t n_slots;          /* reported slots: slots[first_slot .. first_slot + n_slots) */
	uint32_t small_side;       /* junction event: min(split + pos1, split + pos2) - 1 */
	uint32_t large_side;       /*                 max(split + pos1, split + pos2) */
	uint32_t first_slot;
} svg_fragile_window;          /* 28 bytes */

typedef struct svg_fragile_slot {
	uint32_t position;         /* the slot's voting position */
	int16_t  rec[9];           /* indel_recorder[0..8], zero after the first empty section */
	uint16_t _pad;
} svg_fragile_slot;            /* 24 bytes */

typedef struct svg_fragile_result {
	uint64_t n_windows, n_slots;
	svg_fragile_window *windows;   /* (block, read, strand, end, window) order: do_voting's */
	svg_fragile_slot *slots;       /* window by window, each window's in row-major slot order */
} svg_fragile_result;

int  svg_fragile_batch(svg_index *idx, const svg_params *p, const svg_reads *r1, const svg_reads *r2,
                       svg_fragile_result *out);
void svg_fragile_free(svg_fragile_result *r);

/* Per-batch statistics of the last svg_vote_batch* call on this handle
 * (filled only after svg_set_stats(idx,1)); used for the algorithmic-byte roofline. */
typedef struct svg_batch_stats {
	uint64_t probes;             /* gehash_go_X calls                         */
	uint64_t bucket_items;       /* sum of items in the probed buckets        */
	uint64_t hits;               /* sum of equal-key run lengths              */
	uint64_t results;            /* mapping records with selected_votes > 0   */
	uint64_t deferred;           /* single-end align: reads that left the lane-per-read
	                                path and were voted by the wave-per-read kernel */
} svg_batch_stats;
int svg_set_stats(svg_index *idx, int enable);

/* Upper bound of read lengths passed to svg_vote_batch_device on this handle
 * (default 256; svg_vote_batch measures its own batch).  A tighter bound lets
 * the library pick a kernel variant with smaller probe tables and higher
 * occupancy.  A read that needs more subread probes than the bound provides
 * gets zeroed records and raises the handle's sticky device error, which
 * svg_device_status() reports as SVG_E_ARG (svg_vote_batch checks it itself). */
int svg_set_max_read_length(svg_index *idx, int max_len);
/* Waits for the work queued on the handle and returns 0, or SVG_E_ARG (message in
 * svg_last_error) when a read since the previous check violated the read-length
 * bound; clears the error.  Calls on one handle are ordered on the device even
 * when they are given different streams. */
int svg_device_status(svg_index *idx);
int svg_get_stats(const svg_index *idx, svg_batch_stats *out);

/* Per-kernel device time (diagnostics / roofline): while enabled, every probe_kernel
 * and vote_kernel launch is bracketed by HIP events on its stream.  svg_get_timing
 * waits for the last recorded event and returns the summed milliseconds and launch
 * counts since svg_set_timing(idx, 1). */
int svg_set_timing(svg_index *idx, int enable);
int svg_get_timing(svg_index *idx, double *probe_ms, double *vote_ms, int *probe_launches, int *vote_launches);
/* The same per kernel: ms[k] / launches[k] for k = 0 probe_kernel, 1 vote_kernel (wave per
 * read), 2 gather_kernel, 3 lane_kernel (lane per read; single-end align).  vote_ms of
 * svg_get_timing is the sum of kinds 1-3. */
int svg_get_kernel_timing(svg_index *idx, double ms[4], int launches[4]);

const char *svg_last_error(void);
int svg_abi_version(void);
/* Expansion worker threads the host entry points use: the "host_threads" option if set, else
 * the CPUs this process may run on (affinity mask capped by the cgroup CPU quota) divided by
 * LOCAL_WORLD_SIZE (one rank per GPU on the node), clamped to 2..12. */
int svg_host_threads(void);

/* NUMA placement of the host side.  svg_host_placement: the NUMA node of `device`'s
 * PCIe function (-1 unknown) and how many CPUs of that node this process may run on; the host
 * entry points pin their expansion workers to those CPUs (when there are any) and take their
 * pinned staging pages from that node.  svg_host_alloc: pinned host memory whose pages come from
 * the node of idx's GPU -- for the caller's reads and records, which the workers and the copy
 * engines touch at ~100 GB/s per rank; release with svg_host_free.  svg_cpulist_parse parses a
 * sysfs cpulist ("0-15,64-79") into a byte mask of `max` entries and returns the CPUs it set. */
int  svg_host_placement(int device, int *node, int *cpus_on_node);
int  svg_host_alloc(svg_index *idx, size_t bytes, void **out);
void svg_host_free(void *p);
int  svg_cpulist_parse(const char *list, uint8_t *mask, int max);

/*
 * Process-wide implementation options.  The library reads no environment variable of its own
 * (only torchrun's LOCAL_WORLD_SIZE, to size host thread pools): tests and tuning set these
 * explicitly.  No option changes a record -- every setting selects among exact implementations
 * of the same reference behaviour (probe images, kernel paths, chunk and sub-batch sizes, pool
 * sizes) or turns on diagnostics printed to stderr.  Names (value 0 / -1 = the default):
 *   host_threads, host_sub      expansion workers; reads per host sub-batch
 *   chunk, overlap              reads per probe-record chunk; 1/0 force the two-stream chunk pipeline
 *   lane                        1 lane kernels + deferral (default), 2 defer every read to the
 *                               wave kernel, 3 no lane kernels (wave kernel only)
 *   lane_unfused, lane_bin      separate gather kernel; 2 = no count bins
 *   lane_cap, lane_pe_cap, lane_pairs, lane_mid   lane-path capacities (candidates, pairs)
 *   no_bcode, no_khash, khash64, no_bline, no_compact, kinline, khash_probe, probe_v1,
 *   no_window, probe_colmajor   probe images / probe kernel variants picked at index load
 *   wave_cap                    resident wave-kernel blocks per CU beside the next chunk
 *   probe_cap                   probe line kernel grid, blocks per CU (default 32)
 *   wave_cus, lane_cus_excl     CU masks of the device's streams (read when they are created, at
 *                               the first index load): the wave-kernel stream on CUs 0..wave_cus-1,
 *                               the probe / lane stream on the others with lane_cus_excl 1
 *   host_ramp                   host-buffer entries: sub-batches ramped at both ends (default 1)
 *   host_slots                  device slots of the chunk pipeline, 2 (default) or 3
 *   wave_static                 eighths (0-8) of a chunk's deferred reads the wave kernel deals
 *                               out statically before its work counter (default 6 single-end,
 *                               0 pairs)
 *   keys_literal, long_probes   svg_probe_keys / svg_long_vote_batch variants
 *   debug, pipe_debug, long_debug  diagnostics on stderr
 * svg_set_option returns SVG_E_ARG for an unknown name; svg_get_option returns the current value
 * (0 for an unknown name). */
int     svg_set_option(const char *name, int64_t value);
int64_t svg_get_option(const char *name);

/*
 * Index builder (replaces subread-buildindex for a single-block index,
 * index-builder.c:1014-1306): writes <prefix>.00.b.tab/.00.b.array/.reads/
 * .files/.log byte-identical (tab/array/reads) to the reference.
 *   gap 1 = full index (-F), 3 = gapped (default); memory_mb = -M (8000);
 *   force_one_block = -B; repeat_threshold = -f (100).
 */
int svg_build_index(const char *fasta, const char *prefix, int gap, int memory_mb,
                    int force_one_block, int repeat_threshold);

/* Seeded synthetic data for tests/benchmarks (genRandomReads counterpart). */
void svg_sim_genome(char *out, uint64_t length, uint64_t seed);
void svg_sim_repeats(char *genome, uint64_t length, uint64_t n_copies, uint32_t element_len,
                     uint32_t n_families, double divergence, uint64_t seed);
int  svg_sim_reads(const char *genome, const uint64_t *ctg_start, const uint32_t *ctg_len,
                   uint32_t n_ctg, uint64_t first, uint64_t n_reads, int len, double sub,
                   double indel_frac, double n_rate, uint64_t seed, char *seq,
                   uint32_t *truth_ctg, uint32_t *truth_pos, uint8_t *truth_strand, int threads);
/* paired-end fragments (test/bench input generator): R1 forward, R2 reverse
 * complement of the fragment end; pairs first..first+n_pairs-1 of the stream. */
int  svg_sim_pairs(const char *genome, const uint64_t *ctg_start, const uint32_t *ctg_len, uint32_t n_ctg,
                   uint64_t first, uint64_t n_pairs, int len, double ins_mean, double ins_sd, int ins_max,
                   double sub, uint64_t seed, char *seq1, char *seq2, int threads);

#ifdef __cplusplus
}
#endif
#endif /* SUBREAD_VOTE_H */
