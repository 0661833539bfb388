"""Timing-only (WRONG RESULTS) diagnostic builds of the engine, kept out of the product source.

usage: python tools/diag_variant.py NAME [NAME ...]   -> tools/diaglib/libnpfn_NAME.so

Each NAME is a set of text edits applied to a scratch copy of npe-pfn_amd/csrc (under /tmp),
which is then built with the product Makefile.  The product tree never carries a diagnostic
switch; a removed phase's time is the base build's minus the variant's in a
same-GPU A/B (tools/ab_bench.py).  Edits that no longer match the source fail loudly.
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

# name -> [(file under csrc, old text, new text)]
EDITS = {
    # the row kernel without its GELU (the hidden slab goes to W2 as is)
    "nogelu": [("npfn_rowk2.hip", "__device__ __forceinline__ void gelu4(f32x4& h) {\n",
                "__device__ __forceinline__ void gelu4(f32x4& h) {\n  return;\n")],
    # the row kernel without its LayerNorms (statistics and normalisation; the bf16 fragments stay)
    "noln": [("npfn_rowk2.hip", "__device__ __forceinline__ void layer_norm(Acc& x, const float* lnp) {\n",
              "__device__ __forceinline__ void layer_norm(Acc& x, const float* lnp) {\n  return;\n")],
    # the row kernel without its feature attention (the v / k / q products and barriers stay)
    "nofa": [("npfn_rowk2.hip", "  feat_attn_rows<LONG>(smem, C, nrows);\n", "")],
    # the fused mix + sample without its sampling tail (block scan, walk, thread 0's inverse CDF / NLL)
    "mixnotail": [("npfn_kernels.hip", "  bar_sample_row(p, bz, ystats[1], ystats[0], nb, u, red, scan, th, lp);\n  if (threadIdx.x == 0) {\n    feat[(row_offset + r) * ldf + col] = th;",
                   "  th = u;\n  if (threadIdx.x == 0) {\n    feat[(row_offset + r) * ldf + col] = th;")],
    # the fast mix treating every estimator as untranslated (no border translation)
    "mixnotrans": [("npfn_kernels.hip", "    const bool trans = tr.ett != nullptr && tr.ett[e];\n    f32x4 v[NV];",
                    "    const bool trans = false;\n    f32x4 v[NV];")],
    # the fast ensemble mix without the barrier that closes each translated estimator
    "mixnobar": [("npfn_kernels.hip", "__syncthreads();  // pc / scan are rewritten by the next translated estimator",
                  "// (diag: no barrier)")],
}


def build(name: str) -> str:
    if name not in EDITS:
        raise SystemExit(f"unknown variant {name}; known: {sorted(EDITS)}")
    scratch = f"/tmp/npfn_diag_{name}"
    shutil.rmtree(scratch, ignore_errors=True)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(scratch, "include"))
    os.makedirs(os.path.join(scratch, "npe-pfn_amd"))
    shutil.copytree(os.path.join(ROOT, "npe-pfn_amd", "csrc"), os.path.join(scratch, "npe-pfn_amd", "csrc"))
    shutil.copy(os.path.join(ROOT, "npe-pfn_amd", "Makefile"), os.path.join(scratch, "npe-pfn_amd"))
    for fn, old, new in EDITS[name]:
        p = os.path.join(scratch, "npe-pfn_amd", "csrc", fn)
        src = open(p).read()
        if old not in src:
            raise SystemExit(f"variant {name}: edit target not found in {fn}: {old[:60]!r}")
        open(p, "w").write(src.replace(old, new))
    out = os.path.join(ROOT, "tools", "diaglib", f"libnpfn_{name}.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run(["make", "-s", "-C", os.path.join(scratch, "npe-pfn_amd"), f"OUT={out}", "-j4"], check=True)
    return out


if __name__ == "__main__":
    for n in sys.argv[1:]:
        print(build(n))
