#!/usr/bin/env python
"""Scan gfx950 device assembly for the 128-bit-store write-after-read hazard: a buffer/global store of more than
64 bits whose data VGPRs are overwritten by the very next instruction (no wait state). LLVM only guards it for MUBUF
stores whose soffset is not a register; on the MI355X the unguarded form lost store data under load
(csrc/mlp.hip copy_tile_pm). Exit status 1 if any such pair is found.

    python tools/check_store_hazards.py file.s [...]
"""
import re
import sys

# buffer stores name the data VGPRs first; global stores name the 64-bit address first, then the data
STORE = re.compile(r"(?:buffer_store_dwordx(?:3|4) |global_store_dwordx(?:3|4) v\[\d+:\d+\], )v\[(\d+):(\d+)\]")
WRITE = re.compile(r"(v_\S+|ds_read\S*|global_load\S*|buffer_load\S*)\s+v\[?(\d+)(?::(\d+))?")


def scan(path):
    lines = [ln.strip() for ln in open(path) if ln.strip() and not ln.strip().startswith((";", "."))]
    found = []
    n_stores = 0
    for i, ln in enumerate(lines):
        m = STORE.match(ln)
        if not m:
            continue
        n_stores += 1
        a, b = int(m.group(1)), int(m.group(2))
        if i + 1 < len(lines):
            nxt = lines[i + 1]
            w = WRITE.match(nxt)
            if w:
                lo = int(w.group(2))
                hi = int(w.group(3) or lo)
                if not (hi < a or lo > b):
                    found.append(f"{ln}  ->  {nxt}")
    return n_stores, found


def main():
    bad = 0
    for path in sys.argv[1:]:
        n, found = scan(path)
        for f in found:
            print(f"{path}: {f}")
        print(f"{path}: {n} wide stores, {len(found)} with their data VGPRs overwritten by the next instruction")
        bad += len(found)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
