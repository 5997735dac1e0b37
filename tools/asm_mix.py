#!/usr/bin/env python3
"""Instruction mix of the hottest MFMA basic blocks per kernel in a device assembly file (hipcc --cuda-device-only
-S): per block the MFMA count against VALU / LDS / VMEM / SALU / waitcnt counts and the most frequent VALU opcodes.
Development tool: the f32 MFMA shares its issue with the VALU (profiles/r3_probe_mfma_valu*.jsonl), so VALU per MFMA in
the steady-state loops is a cost.
    python tools/asm_mix.py FILE.s [kernel-substring] [blocks-per-kernel]"""
import collections
import re
import sys


def main():
    path = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "mlp_"
    nb = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    lines = open(path).read().split("\n")
    func, blocks, cur = None, collections.defaultdict(list), None
    for ln in lines:
        m = re.match(r"^(_ZN6yanerf\w+):", ln)
        if m:
            func, cur = m.group(1), (m.group(1), "entry")
            continue
        m = re.match(r"^(\.LBB\d+_\d+):", ln)
        if m and func:
            cur = (func, m.group(1))
            continue
        if func and ln.startswith("\t") and cur:
            t = ln.strip()
            if t and not t.startswith((".", ";")):
                blocks[cur].append(t.split()[0])
    by_func = collections.defaultdict(list)
    for (f, b), ins in blocks.items():
        by_func[f].append((sum(i.startswith("v_mfma") for i in ins), b, ins))
    for f, bl in by_func.items():
        if sub not in f:
            continue
        print(f[:90])
        for nm, b, ins in sorted(bl, reverse=True)[:nb]:
            if nm == 0:
                continue
            c = collections.Counter()
            for i in ins:
                k = ("mfma" if i.startswith("v_mfma") else "valu" if i.startswith("v_") else "lds" if i.startswith("ds_")
                     else "vmem" if i.startswith(("global_", "buffer_")) else "wait" if i.startswith("s_waitcnt")
                     else "barrier" if i.startswith("s_barrier") else "salu" if i.startswith("s_") else "other")
                c[k] += 1
            vc = collections.Counter(i for i in ins if i.startswith("v_") and not i.startswith("v_mfma"))
            print(f"  {b}: {dict(c)}  valu/mfma={c['valu'] / max(1, c['mfma']):.2f}  top: {vc.most_common(6)}")


if __name__ == "__main__":
    main()
