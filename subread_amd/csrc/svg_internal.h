/* svg_internal.h -- host-side internals shared by the C host code and the HIP code. */
#ifndef SVG_INTERNAL_H
#define SVG_INTERNAL_H
#include <stdint.h>
#include "subread_vote.h"

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
void svg_host_index_free(svg_host_index *ix);

uint32_t svg_bucket_count(uint64_t expected_items, int gap);

#ifdef __cplusplus
}
#endif
#endif
