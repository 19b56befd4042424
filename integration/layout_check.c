/*
 * integration/layout_check.c -- compile-time proof that the boundary records are the
 * reference's records: every field of svg_mapping_result / svg_subjunc_result
 * (include/subread_vote.h) has the size and offset of the same field of
 * mapping_result_t (core.h:350-370) / subjunc_result_t (core.h:397-410), and the
 * constants match subread.h / core.h.  Compiled by tests/test_boundary_ref.py against
 * the reference's own headers (gcc -c -I/root/reference/src -Iinclude).
 */
#include <stddef.h>
#include "subread.h"
#include "core.h"
#include "subread_vote.h"

#define SAME(T1, T2, f1, f2) \
	_Static_assert(offsetof(T1, f1) == offsetof(T2, f2), #f1 " offset"); \
	_Static_assert(sizeof(((T1 *)0)->f1) == sizeof(((T2 *)0)->f2), #f1 " size")

_Static_assert(sizeof(svg_mapping_result) == sizeof(mapping_result_t), "mapping_result_t size");
SAME(svg_mapping_result, mapping_result_t, selected_position, selected_position);
SAME(svg_mapping_result, mapping_result_t, result_flags, result_flags);
SAME(svg_mapping_result, mapping_result_t, read_length, read_length);
SAME(svg_mapping_result, mapping_result_t, selected_votes, selected_votes);
SAME(svg_mapping_result, mapping_result_t, used_subreads_in_vote, used_subreads_in_vote);
SAME(svg_mapping_result, mapping_result_t, noninformative_subreads_in_vote, noninformative_subreads_in_vote);
SAME(svg_mapping_result, mapping_result_t, indels_in_confident_coverage, indels_in_confident_coverage);
SAME(svg_mapping_result, mapping_result_t, is_fully_covered, is_fully_covered);
SAME(svg_mapping_result, mapping_result_t, selected_indel_record, selected_indel_record);
SAME(svg_mapping_result, mapping_result_t, confident_coverage_start, confident_coverage_start);
SAME(svg_mapping_result, mapping_result_t, confident_coverage_end, confident_coverage_end);
SAME(svg_mapping_result, mapping_result_t, subread_quality, subread_quality);

_Static_assert(sizeof(svg_subjunc_result) == sizeof(subjunc_result_t), "subjunc_result_t size");
SAME(svg_subjunc_result, subjunc_result_t, split_point, split_point);
SAME(svg_subjunc_result, subjunc_result_t, minor_votes, minor_votes);
SAME(svg_subjunc_result, subjunc_result_t, double_indel_offset, double_indel_offset);
SAME(svg_subjunc_result, subjunc_result_t, indel_at_junction, indel_at_junction);
SAME(svg_subjunc_result, subjunc_result_t, small_side_increasing_coordinate, small_side_increasing_coordinate);
SAME(svg_subjunc_result, subjunc_result_t, large_side_increasing_coordinate, large_side_increasing_coordinate);
SAME(svg_subjunc_result, subjunc_result_t, minor_position, minor_position);
SAME(svg_subjunc_result, subjunc_result_t, minor_coverage_start, minor_coverage_start);
SAME(svg_subjunc_result, subjunc_result_t, minor_coverage_end, minor_coverage_end);

_Static_assert(SVG_MAX_READ_LENGTH == MAX_READ_LENGTH, "MAX_READ_LENGTH");
_Static_assert(SVG_MAX_INDEL_SECTIONS == MAX_INDEL_SECTIONS, "MAX_INDEL_SECTIONS");
_Static_assert(SVG_VOTE_TABLE_SIZE == GENE_VOTE_TABLE_SIZE, "GENE_VOTE_TABLE_SIZE");
_Static_assert(SVG_VOTE_SPACE == GENE_VOTE_SPACE, "GENE_VOTE_SPACE");
_Static_assert(SVG_NEGATIVE_STRAND_FLAG == CORE_IS_NEGATIVE_STRAND, "CORE_IS_NEGATIVE_STRAND");
/* gene_vote_number_t is the reference's vote counter type (short) */
_Static_assert(sizeof(gene_vote_number_t) == sizeof(int16_t), "gene_vote_number_t");
