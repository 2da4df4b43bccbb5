"""Build-time hazard lint of the gfx950 code objects (tools/isa_lint.py): no
VALU write of an MFMA SrcA/SrcB VGPR within 2 wait states of the MFMA.  The
matrix-core GP (csrc/kf_gp_mfma.h) has no inline assembly left, so the
compiler's hazard recognizer owns every such pad; this test checks its
output, and that the lint itself catches a missing pad."""
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))

import isa_lint  # noqa: E402

LISTING = """
0000000000001000 <kern>:
\tv_exp_f32_e32 v64, v64
\tv_cvt_pkrtz_f16_f32 v62, v64, v65
\tv_fma_mixhi_f16 v66, v62, s0, v70 op_sel:[1,0,0] op_sel_hi:[1,0,0]
\t{pad}
\tv_mfma_f32_32x32x16_f16 v[30:45], v[86:89], v[66:69], v[30:45]
"""


@pytest.mark.parametrize("pad,ok", [("", False), ("s_nop 0", False), ("s_nop 1", True),
                                    ("v_add_f32_e32 v1, v2, v3\n\tv_add_f32_e32 v4, v5, v6", True)])
def test_lint_flags_missing_wait_states(pad, ok):
    insts = isa_lint.parse(LISTING.format(pad=pad))
    bad = isa_lint.lint_listing(insts, "t")
    assert (not bad) == ok, bad


def test_built_code_objects_have_no_mfma_operand_hazards():
    sos = sorted((ROOT / "kafka_inferenceengine_amd").glob("_kafka_hip*.so"))
    if not sos or not isa_lint.OBJDUMP.exists():
        pytest.skip("extension not built or llvm-objdump missing")
    for so in sos:
        n, bad = isa_lint.lint_so(so)
        assert n > 0, f"{so.name}: no MFMA instructions found (matrix-core GP not compiled?)"
        assert not bad, bad[:5]


# Hot kernels and their register budget: >= 3 waves per SIMD (<= 168 VGPRs)
# and no scratch.  A regression here cost round 3 a 1.3x slower headline
# before it was caught (row addresses hoisted out of the fused GN loop:
# 256 VGPRs, one wave per SIMD).
HOT = {   # kernel: (min waves per SIMD, max scratch bytes per lane)
    "_ZN2kf20analysis_mfma_kernelILi7ELi4ELi2ELi256ELi3ELi1ELb1ELi1EEEvNS_12AnalysisArgsE": (3, 0),   # tip7 headline (TIP layout, fused forecast)
    "_ZN2kf20analysis_mfma_kernelILi7ELi4ELi2ELi256ELi3ELi1ELb1ELi2EEEvNS_12AnalysisArgsE": (3, 0),   # spatial (+ regulariser prepare)
    "_ZN2kf20analysis_mfma_kernelILi7ELi4ELi2ELi256ELi3ELi1ELb1ELi3EEEvNS_12AnalysisArgsE": (3, 0),   # small emulators (next group's forecast inputs ahead)
    "_ZN2kf20analysis_mfma_kernelILi7ELi4ELi2ELi256ELi3ELi1ELb1ELi0EEEvNS_12AnalysisArgsE": (3, 0),   # generic TIP layout (first date)
    "_ZN2kf20analysis_mfma_kernelILi7ELi4ELi2ELi256ELi3ELi1ELb0ELi0EEEvNS_12AnalysisArgsE": (3, 0),   # block-by-block variant (A/B)
    "_ZN2kf20analysis_mfma_kernelILi7ELi4ELi2ELi256ELi3ELi0ELb0ELi0EEEvNS_12AnalysisArgsE": (3, 0),   # runtime band layout
    "_ZN2kf15analysis_kernelILi7ELi4ELi2ELi4ELb0EEEvNS_12AnalysisArgsE": (3, 0),           # TIP VALU loop
    "_ZN2kf15analysis_kernelILi7ELin2ELi4ELi4ELb0EEEvNS_12AnalysisArgsE": (3, 0),          # identity7 (bf16 y)
    # PROSAIL (55-float packed A per lane): 2 waves/SIMD, no scratch since the
    # epilogue stores use SGPR row bases (kf_core.h pxp; was 36 B, 2.5 % slower)
    "_ZN2kf22analysis_mfma_g_kernelILi10ELi10ELi2ELb0ELb0ELi0EEEvNS_12AnalysisArgsE": (2, 0),
    "_ZN2kf22analysis_mfma_g_kernelILi10ELi10ELi2ELb0ELb1ELi0EEEvNS_12AnalysisArgsE": (2, 0),
    "_ZN2kf22analysis_mfma_g_kernelILi10ELi10ELi2ELb0ELb1ELi1EEEvNS_12AnalysisArgsE": (2, 0),   # prosail10 (fused forecast)
    # JRC-TIP gain form: 3 waves per SIMD by launch bound, a few registers spilled (measured faster than 2 waves)
    "_ZN2kf16gain_mfma_kernelILi7ELi4ELi2EEEvNS_8GainArgsE": (3, 80),
}


def test_hot_kernels_keep_their_occupancy():
    so = ROOT / "kafka_inferenceengine_amd" / "_kafka_hip.cpython-310-x86_64-linux-gnu.so"
    if not so.exists() or not isa_lint.READELF.exists():
        pytest.skip("extension not built or llvm-readelf missing")
    res = isa_lint.kernel_resources(so)
    for name, (min_waves, max_scratch) in HOT.items():
        assert name in res, f"{name} not in the code objects"
        r = res[name]
        w = isa_lint.waves_per_simd(r["vgpr"], r.get("agpr", 0))
        assert w >= min_waves, (name, r, w)
        assert r["scratch"] <= max_scratch, (name, r)
