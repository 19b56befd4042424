"""CPU: the drop-in boundary checked by a compiler against the REFERENCE's own headers.

* integration/layout_check.c: _Static_assert that every field of svg_mapping_result /
  svg_subjunc_result has the offset and size of the same field of mapping_result_t
  (core.h:350-370) / subjunc_result_t (core.h:397-410), and that the constants match
  subread.h / core.h;
* integration/do_voting_gpu.c: the reference-side binding INTEGRATION.md shows (the
  do_voting replacement) compiles against core.h / core-indel.h / core-junction.h and
  include/subread_vote.h.
Runs where the reference sources exist (this container); skipped elsewhere."""
import os
import subprocess

import pytest

from tests.common import ROOT

REF_SRC = "/root/reference/src"
pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(REF_SRC, "core.h")),
                                reason="reference headers not present")


def _cc(src, tmp_path):
    out = tmp_path / (os.path.basename(src) + ".o")
    r = subprocess.run(["gcc", "-std=gnu11", "-Wall", "-Werror", "-Wno-unused-function", "-c", "-o", str(out),
                        "-I" + REF_SRC, "-I" + os.path.join(ROOT, "include"), "-DMAKE_FOR_EXON", "-DMAKE_STANDALONE",
                        os.path.join(ROOT, src)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out


def test_record_layout_matches_reference_structs(tmp_path):
    _cc("integration/layout_check.c", tmp_path)


def test_integration_stub_compiles_against_reference(tmp_path):
    o = _cc("integration/do_voting_gpu.c", tmp_path)
    syms = subprocess.run(["nm", str(o)], capture_output=True, text=True).stdout
    for s in ("do_voting_gpu", "svg_attach"):
        assert " T " + s in syms
    for s in ("svg_vote_batch_packed", "svg_pack_reads", "svg_index_open", "fetch_next_read_pair", "find_new_indels"):
        assert " U " + s in syms


def test_layout_check_catches_a_wrong_layout(tmp_path):
    bad = tmp_path / "bad.c"
    bad.write_text('#include <stddef.h>\n#include "subread.h"\n#include "core.h"\n#include "subread_vote.h"\n'
                   '_Static_assert(offsetof(svg_mapping_result, confident_coverage_start) == '
                   'offsetof(mapping_result_t, confident_coverage_end), "x");\n')
    r = subprocess.run(["gcc", "-std=gnu11", "-c", "-o", str(tmp_path / "bad.o"), "-I" + REF_SRC,
                        "-I" + os.path.join(ROOT, "include"), str(bad)], capture_output=True, text=True)
    assert r.returncode != 0
