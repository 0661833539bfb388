"""VALU / MFMA instruction budget of one kernel instance attributed to the source phase each
instruction comes from (debug line tables with the inline chain), loops weighted by trip counts.

    hipcc --offload-arch=gfx950 -O3 -g <the Makefile's flags> --cuda-device-only -c npfn_rowk2.hip -o rk.o
    clang-offload-bundler --unbundle --type=o --input=rk.o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=rk.co
    python tools/isa_phases.py rk.co <mangled kernel symbol> [--trips loop=N ...] [--list-loops]

Without --trips every loop counts once; --list-loops prints each loop (a backward branch) with its
source location and static size so the trips can be given by that location (e.g.
--trips npfn_rowk2.hip:624=10).  Phases (first match along the inline chain): feature attention
(feat_attn_rows*, read_vt and the LDS image writes of feat_pair), GELU, LayerNorm, bf16 operand
conversion (to_frag / pack8 / pack_bf2 outside the above), row stores, weight-ring barrier + DMA
(Ring), chunk pipeline (run_chunk / run_s / run_o / read_frag: the MFMAs, fragment reads and their
addressing), tile setup (the rest).
"""
import argparse
import re
import subprocess
from collections import Counter, defaultdict

LLVM = "/opt/rocm/lib/llvm/bin"


def klass(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(("v_", "ds_swizzle", "ds_bpermute")) and not op.startswith("v_accvgpr"):
        if re.match(r"v_(exp|log|rcp|rsq|sqrt|sin|cos)_", op):
            return "valu:trans"
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("s_"):
        return "salu"
    return "other"


def phase(chain):
    names = [c[0] for c in chain]
    txt = " | ".join(names)
    if re.search(r"feat_attn_rows|read_vt", txt):
        return "feature attention"
    if "feat_pair" in txt and not re.search(r"run_chunk|run_o|run_s|read_frag|read_window|Ring::", txt):
        return "feature attention"
    if re.search(r"gelu", txt) and not re.search(r"run_chunk[^|]*$", names[0]):
        if re.search(r"gelu4|gelu_tanh", txt):
            return "GELU"
    if re.search(r"layer_norm|ln_stats|ln_coef|ln_norm", txt):
        return "LayerNorm"
    if re.search(r"to_frag|pack8|pack_bf2", txt) and "store_bf16_row" not in txt:
        return "bf16 conversion"
    if re.search(r"store_bf16_row|store_f32_row", txt):
        return "row stores"
    if "Ring::" in txt:
        return "ring barrier + DMA"
    if re.search(r"run_chunk|run_s|run_o|read_frag|read_window|run_w2_gelu", txt):
        return "chunk pipeline"
    return "tile setup / other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("co")
    ap.add_argument("symbol")
    ap.add_argument("--trips", nargs="*", default=[])
    ap.add_argument("--list-loops", action="store_true")
    a = ap.parse_args()
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", a.co], capture_output=True,
                         text=True, check=True).stdout.split("\n")
    st = next(i for i, l in enumerate(dis) if l.endswith(f"<{a.symbol}>:"))
    ins = []
    for l in dis[st + 1:]:
        if not l.strip():
            if ins:
                break
            continue
        m = re.match(r"\s*(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):(.*)$", l)
        if not m:
            continue
        ins.append((int(m.group(3), 16), m.group(1), m.group(4)))
        if m.group(1) == "s_endpgm":
            break
    addrs = "\n".join(hex(x[0]) for x in ins)
    sym = subprocess.run([f"{LLVM}/llvm-symbolizer", f"--obj={a.co}", "--inlining"], input=addrs,
                         capture_output=True, text=True, check=True).stdout.strip().split("\n\n")
    chains = []
    for blk in sym:
        ls = blk.strip().split("\n")
        chains.append([(ls[i], ls[i + 1].split("/")[-1]) for i in range(0, len(ls) - 1, 2)])
    idx = {addr: i for i, (addr, _, _) in enumerate(ins)}
    loops = []
    for i, (addr, op, opnd) in enumerate(ins):
        if op.startswith("s_cbranch") or op == "s_branch":
            m = re.search(r"<[^+>]*\+0x([0-9a-fA-F]+)>", opnd)
            tgt = ins[0][0] + int(m.group(1), 16) if m else None
            if tgt is not None and tgt in idx and idx[tgt] <= i:
                loops.append((idx[tgt], i))
    # a loop = a head with every backward branch to it (a rotated or multi-exit loop has several):
    # the span from the head to its last branch
    last = {}
    for s_, e_ in loops:
        last[s_] = max(last.get(s_, e_), e_)
    loops = sorted(last.items(), key=lambda r: r[1] - r[0])
    trips = dict(t.split("=") for t in a.trips)
    weight = [1.0] * len(ins)
    for (s, e) in loops:
        loc = chains[e][0][1] if chains[e] else "?"
        loc_head = chains[s][0][1] if chains[s] else "?"
        key = next((k for k in trips if k == str(s) or loc_head.startswith(k)), None)
        t = float(trips[key]) if key else 1.0
        if a.list_loops:
            inner = Counter(phase(chains[j]) for j in range(s, e + 1))
            print(f"loop [{s}, {e}] {e - s + 1} instrs, head {loc_head}, trips {t:g}: "
                  + ", ".join(f"{k} {v}" for k, v in inner.most_common(3)))
        for j in range(s, e + 1):
            weight[j] *= t
    tab = defaultdict(Counter)
    for (addr, op, _), ch, w in zip(ins, chains, weight):
        tab[phase(ch)][klass(op)] += w
    tot = Counter()
    for c in tab.values():
        tot.update(c)
    mf = tot["mfma"] or 1.0
    valu = tot["valu"] + tot["valu:trans"]
    print(f"{a.symbol}: {len(ins)} static instructions, {len(loops)} loops")
    print(f"{'phase':22s} {'VALU':>9s} {'(trans)':>8s} {'VALU/MFMA':>10s} {'share':>7s} {'MFMA':>8s} {'LDS':>7s} {'SALU':>7s}")
    for ph, c in sorted(tab.items(), key=lambda kv: -(kv[1]["valu"] + kv[1]["valu:trans"])):
        v = c["valu"] + c["valu:trans"]
        print(f"{ph:22s} {v:9.0f} {c['valu:trans']:8.0f} {v / mf:10.3f} {v / max(valu, 1):7.1%} {c['mfma']:8.0f} "
              f"{c['lds']:7.0f} {c['salu']:7.0f}")
    print(f"{'total':22s} {valu:9.0f} {tot['valu:trans']:8.0f} {valu / mf:10.3f} {'':7s} {tot['mfma']:8.0f} "
          f"{tot['lds']:7.0f} {tot['salu']:7.0f}")


if __name__ == "__main__":
    main()
