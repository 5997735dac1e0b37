"""Register the package directory `yet-another-nerf_amd/` under the importable name `yanerf_amd`.

The package directory name contains hyphens (repo layout contract), which Python cannot
`import` directly; importing this module once makes `import yanerf_amd` work.
"""
import importlib.util
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent / "yet-another-nerf_amd"


def load():
    if "yanerf_amd" in sys.modules:
        return sys.modules["yanerf_amd"]
    spec = importlib.util.spec_from_file_location(
        "yanerf_amd", PKG_DIR / "__init__.py", submodule_search_locations=[str(PKG_DIR)]
    )
    mod = importlib.util.module_from_spec(spec)
    sys.modules["yanerf_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


load()
