"""Register, spill and scratch budget of every gfx950 kernel in libbsgp.so
(CPU only: reads the built code objects' metadata, tools/kernel_meta.py).

Two silent regressions of round 5 (C3 -9 %, C4 -15 %) were scratch memory:
a lambda's by-reference captures or a plan copy living on the private stack
of a hot kernel.  Every kernel must have no VGPR spills and no private
segment unless it is on the allow-list below, and an allow-listed kernel must
stay at or under its budget.  What each allowance is:

* persistent solvers (k_persist, three builds): the phase functions are
  noinline calls, so their private segment is the largest
  phase's frame plus the kernel's own frame of at most 36 B (the spills
  counted here: 64-bit values the kernel keeps across the calls).  A phase
  frame is the callee-saved VGPRs it clobbers (v40-47, v56-63, ... up to its
  register count: 64 at 168 VGPRs) and the whole-wave VGPRs holding its SGPR
  spills, saved at entry and restored at exit once per phase call, plus that
  phase's own spill slots: C3's line search 3 (12 B), the folded setup 14
  (it is a 188-VGPR kernel squeezed to the solver's 168; it runs once per
  image).  C3's kernel: setup 344 B + 32 = 376 B; line search 292 B.
* the cooperative (512-thread, 2 waves/SIMD) line search k_ls<.., COOP>:
  2-41 VGPR spills at the 256-VGPR cap (C4's phase kernels).
* the per-wave phase line search k_ls<..> and k_setup<false, ..> (and the
  256-thread cooperative k_setup<true, ..>, off the bench paths): a 36-B
  frame that no instruction of the kernel addresses (no scratch_* or
  buffer access in its code; checked in the ISA, profiles/r06/regbudget.txt).
* psf_stamps_kernel: the DIAPL coefficient arrays of one stamp (runs once
  per PSF model, off the solver path).
Everything else has none.  k_setup carried a 1000-B frame until round 6
(np_f32_sum, an out-of-line template, took the Team and its lambda captures
to the stack): now under the 36-B allowance above.
"""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
LIB = os.path.join(ROOT, "beta-sgp_amd", "libbsgp.so")

# (kernel-name regex, max VGPR spills, max private segment bytes)
ALLOW = [
    (r"^_ZN4bsgp9k_persistILb0ELi2ELi3ELb0EdLb1E", 10, 376),   # C3's timed kernel
    (r"^_ZN4bsgp9k_persistILb0ELi\d+ELi(0|3|4|n1)ELb0E[df]Lb[01]E", 10, 380),
    (r"^_ZN4bsgp9k_persistILb0ELi1ELin1ELb1E[df]Lb0E", 10, 640),  # adaptive beta
    (r"^_ZN8bsgp_app9k_persist", 1, 544),
    (r"^_ZN9bsgp_c5129k_persist", 1, 532),
    (r"^_ZN9bsgp_c5124k_lsILi\d+ELi(3|4)ELb0ELb1E", 6, 20),
    (r"^_ZN9bsgp_c5124k_lsILi1ELin1ELb1ELb1E", 41, 144),
    (r"^_ZN4bsgp4k_lsILi\d+ELi(0|3|4|n1)ELb0ELb0E[df]", 0, 36),
    (r"^_ZN4bsgp7k_setupILb0E[df]", 0, 36),
    # the 256-thread cooperative setup (only when BSGP_COOP512 is off; the
    # cooperative plans run bsgp_c512::k_setup): the same unaddressed 36-B frame
    (r"^_ZN4bsgp7k_setupILb1E[df]", 0, 36),
    # C4's cooperative setup (once per solve): the same unaddressed 36-B frame
    # since round 6's DPP / swizzle wave reductions (checked in the ISA: no
    # scratch or buffer instruction in the kernel)
    (r"^_ZN9bsgp_c5127k_setupILb1E[df]", 0, 36),
    (r"^_ZN4bsgp17psf_stamps_kernel", 0, 816),
]

# the kernels bench.py's headline and the C4 line run: never any spill
HOT_NO_SPILL = [r"^_ZN4bsgp5k_col",
                r"^_ZN9bsgp_c5125k_col", r"^_ZN9bsgp_c5125k_dir", r"^_ZN9bsgp_c5124k_bb"]


@pytest.fixture(scope="module")
def meta():
    assert os.path.exists(LIB), "libbsgp.so not built (run __graft_entry__.build())"
    import kernel_meta
    m = kernel_meta.kernels(LIB)
    assert len(m) > 100, f"only {len(m)} kernels found in {LIB}"
    return m


def _budget(name):
    for pat, sp, pr in ALLOW:
        if re.search(pat, name):
            return sp, pr
    return 0, 0


def test_every_kernel_within_its_spill_and_scratch_budget(meta):
    bad = []
    for name, m in sorted(meta.items()):
        sp, pr = _budget(name)
        if m["vgpr_spill"] > sp or m["private"] > pr or m["dyn_stack"]:
            bad.append(f"{name}: spills {m['vgpr_spill']} (<= {sp}), private {m['private']} B "
                       f"(<= {pr}), dynamic stack {m['dyn_stack']}")
    assert not bad, "kernels over their budget:\n" + "\n".join(bad)


def test_hot_kernels_have_no_scratch(meta):
    for pat in HOT_NO_SPILL:
        hits = [n for n in meta if re.search(pat, n)]
        assert hits, pat
        for n in hits:
            assert meta[n]["vgpr_spill"] == 0 and meta[n]["private"] == 0, (n, meta[n])


def test_timed_kernel_frame_is_callee_saves_only(meta):
    """C3's k_persist<false, 2, 3, false, double, true>: 3 waves per SIMD, and
    a private segment no larger than the callee-saved set of a 168-VGPR phase
    (64 VGPRs + 4 SGPR-spill VGPRs = 272 B) plus the folded setup's 14 spill
    slots and alignment (344 B), plus the kernel's own 32 B."""
    n = [k for k in meta if k.startswith("_ZN4bsgp9k_persistILb0ELi2ELi3ELb0EdLb1E")]
    assert len(n) == 1
    m = meta[n[0]]
    assert m["vgpr"] <= 168
    assert m["private"] <= 344 + 32, m
