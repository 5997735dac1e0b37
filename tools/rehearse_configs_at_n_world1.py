#!/usr/bin/env python
"""One-card rehearsal of bench.configs_at_n -- the legs the driver's N > 1 runs add (BASELINE configs[3] Fern fp32 /
bf16 and configs[4] Lego bf16 64 + 256) -- over RCCL at world size 1 (YANERF_PG_AT_WORLD1: the N-rank step schedule
with its two bucketed all-reduces, bf16's coarse bucket started on the side stream beside the fine forward), against
the same legs without a process group. RCCL takes one card per rank, so this is as close to the N-rank path as one
card gets (two ranks on a card need gloo, whose host-side all-reduce dominates a 1 ms step). Development tool (GPU).

    python tools/rehearse_configs_at_n_world1.py pg|plain      -> one JSON line
"""
import json
import math
import os
import sys
from pathlib import Path

mode = sys.argv[1] if len(sys.argv) > 1 else "pg"
for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29561"), ("RANK", "0"), ("WORLD_SIZE", "1"),
             ("LOCAL_RANK", "0")):
    os.environ.setdefault(k, v)
if mode == "pg":
    os.environ["YANERF_PG_AT_WORLD1"] = "1"
sys.argv = sys.argv[:1]
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from yanerf_amd import parallel  # noqa: E402
from yanerf_amd.utils.config import Config  # noqa: E402


def main():
    rank, world, local = parallel.init_distributed()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    cfg = Config.fromfile(str(bench.yanerf_boot.PKG_DIR / "configs/nerf/lego.yml"))
    pcfg = cfg.pipeline
    image = torch.rand(1, 800, 800, 3, generator=torch.Generator().manual_seed(42)).to(dev)
    poses = torch.stack([torch.from_numpy(bench.synthetic_pose(th, -30.0)) for th in np.linspace(-180, 180, 40,
                                                                                                  endpoint=False)]).to(dev)
    focal = torch.tensor([0.5 * 800 / math.tan(0.5 * 0.6911112)], device=dev)
    out = bench.configs_at_n(pcfg, cfg, dev, poses, focal, image, world, steps=20, warmup=5)
    out["mode"] = mode
    out["process_group"] = (torch.distributed.get_backend() if parallel.is_dist() else None)
    print(json.dumps(out))
    if parallel.is_dist():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
