"""Run the reference's standalone loop with the GPU aggregate, unchanged.

    cd <reference>/src
    python -m mfl_amd.launch main_fedavg.py --gpu 0 --dataset mnist --model lr ...

(with the repo root on ``PYTHONPATH`` so ``mfl_amd`` imports).  This imports
the reference's ``fedavg_trainer`` module from the script's directory,
replaces ``FedAvgTrainer.aggregate`` (fedavg_trainer.py:441) with the HIP
drop-in via :func:`mfl_amd.install`, then executes the script as
``__main__`` -- ``main_fedavg.py``'s own ``from fedavg_trainer import
FedAvgTrainer`` (main_fedavg.py:16) then binds the patched class, and the round
loop (fedavg_trainer.py:217 ``w_glob = self.aggregate(w_locals)``) runs on the
GPU with no edit to the reference.
"""
from __future__ import annotations

import importlib
import runpy
import sys
from pathlib import Path


def patch_reference(script_dir: Path, module: str = "fedavg_trainer", cls: str = "FedAvgTrainer"):
    if str(script_dir) not in sys.path:
        sys.path.insert(0, str(script_dir))
    mod = importlib.import_module(module)
    from . import install

    return install(getattr(mod, cls))


def main(argv=None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        raise SystemExit("usage: python -m mfl_amd.launch <main_fedavg.py> [args...]")
    script = Path(argv[0]).resolve()
    patch_reference(script.parent)
    sys.argv = [str(script), *argv[1:]]
    runpy.run_path(str(script), run_name="__main__")


if __name__ == "__main__":
    main()
