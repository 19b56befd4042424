/* svg_internal.h -- host-side internals shared by the C host code and the HIP code. */
#ifndef SVG_INTERNAL_H
#define SVG_INTERNAL_H
#include <stdint.h>
#include "subread_vote.h"
#include "subread_events.h"
#include "subread_realign.h"

#ifdef __cplusplus
extern "C" {
#endif

/* thread-local last-error text (svg_last_error) */
void svg_set_error(const char *fmt, ...);

/* Host image of a single-block base-space index (gehash_t + gene_value_index_t
 * + gene_offset_t of the reference), flattened for upload to HBM:
 *   bstart[nb+1]  item offset of each bucket (u32: items <= 2^32-1, gehash_load
 *                 sorted-hashtable.c:1460)
 *   keys[items]   i16 key_hi = key / nb, bucket order
 *   vals[items]   u32 linear positions, same order
 */
typedef struct svg_host_index {
	uint32_t nb;
	uint64_t items;
	int32_t gap, padding;
	uint32_t *bstart;
	int16_t *keys;
	uint32_t *vals;
	uint32_t start_point, length, start_base_offset, values_bytes;
	uint8_t *values;
	uint32_t n_chr;
	uint32_t *chr_end;       /* .reads offsets (gene_offset_t.read_offsets) */
	char (*chr_name)[200];
	void *map;               /* mmap of the .tab while loading */
	size_t map_len;
} svg_host_index;

int  svg_host_index_load(const char *prefix, svg_host_index *out, int threads);
int  svg_host_index_load_block(const char *prefix, int block, svg_host_index *out, int threads);
int  svg_index_count_blocks(const char *prefix);
/* streaming load (svg_vote.hip): the .tab mapped and its header parsed; the .array / .reads */
int  svg_tab_map(const char *fn, svg_host_index *ix, const uint8_t **first);
int  svg_host_index_load_meta(const char *prefix, int block, svg_host_index *ix);
void svg_host_index_free(svg_host_index *ix);

uint32_t svg_bucket_count(uint64_t expected_items, int gap);

/* host copy (or a wrap, owned = 0) of the index's base arrays and contig table
 * (subread_events.h svg_genome_arrays_open / subread_realign.h svg_genome_arrays_wrap) */
#define SVG_CHR_NAME_LEN 200   /* MAX_CHROMOSOME_NAME_LEN */
typedef struct {
	uint32_t start_point, length, start_base_offset, values_bytes;
	uint8_t *values;
} garray;
struct svg_genome_arrays {
	int nblocks;
	garray *blk;
	uint32_t n_chr;
	uint32_t *chr_end;
	char *chr_name;        /* n_chr x SVG_CHR_NAME_LEN */
	int padding;
	int gap;               /* index_gap of the first table (1 full, 3 gapped): GENE_SLIDING_STEP */
	int owned;             /* the value arrays are freed with the image */
};

/* normalised genome (check_and_convert_FastA semantics, index-builder.c:789-992) */
typedef struct svg_contig {
	char name[200];
	uint64_t start;      /* into bases */
	uint32_t len;
} svg_contig;
typedef struct svg_genome {
	char *bases;         /* A/C/G/T only, contigs concatenated */
	uint64_t nbases, cap;
	svg_contig *ctg;
	uint32_t nctg, ctg_cap;
} svg_genome;
int  svg_genome_read_fasta(const char *path, svg_genome *g);
int  svg_genome_from_mem(const char *const *names, const char *const *seqs, const uint64_t *lens, uint32_t n, svg_genome *g);
void svg_genome_free(svg_genome *g);
/* linear coordinates: O[c] (first base of contig c), windows per contig, index budget */
void svg_genome_layout(const svg_genome *g, int gap, uint64_t *O, uint64_t *nwin);
uint64_t svg_items_budget(int gap, int memory_mb, int force_one_block);
/* writers of the reference on-disk format */
int svg_write_tab(const char *prefix, uint32_t nb, uint64_t items, int gap, const uint32_t *bstart,
                  const int16_t *keys, const uint32_t *vals);
int svg_write_array_reads(const char *prefix, const svg_genome *g, const uint64_t *O, int gap,
                          uint64_t nwin, uint64_t items, uint32_t nb, const char *source);
/* 2-bit LSB-first .array image (gvindex_set), length/values_bytes as gvindex_load sees them */
uint8_t *svg_pack_array(const svg_genome *g, const uint64_t *O, uint32_t *length, uint32_t *values_bytes);

#ifdef __cplusplus
}
#endif
#endif
