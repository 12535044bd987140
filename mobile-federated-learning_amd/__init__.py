"""MI355X-native FedAvg server-side weighted reduction (drop-in for the
reference's ``FedAvgTrainer.aggregate``, src/fedavg_trainer.py:441-458).

Importable as ``mfl_amd`` (see ``/mfl_amd.py`` at the repo root; the
directory name itself is not a Python identifier).

Layers:
  csrc/fedavg_reduce.hip   gfx950 kernels + C ABI (include/fedavg_amd.h)
  _lib                     ctypes binding, fails loudly if the .so is missing
  reduce                   device-resident entry points (torch tensors in HBM)
  layout                   state_dict <-> packed [K, ld] client-major buffers
  aggregate                the drop-in (DeviceAggregator, install, mixin)
  session                  streaming rounds: pack + upload each client as it arrives
  distributed              P-sharded multi-GPU reduce + RCCL all-gather
  multi                    one process, N GPUs: host rounds by columns over N PCIe links
  fpf                      FPF2 bookkeeping (local_w_diffs / A_mat / G_mat) in HBM
"""
from ._lib import FedAvgLibraryError, library_path
from .aggregate import (
    DeviceAggregator,
    FedAvgAggregateMixin,
    aggregate,
    client_arena,
    client_distances,
    estimate_delta,
    default_aggregator,
    install,
    sample_weights,
)
from .layout import KeyTable, ShapeMismatchError, result_dtype
from .reduce import ALIGN_ELEMS, client_sqdist, reduce_packed, reduce_tensors, reduce_with_sqdist, weights_tensor
from .session import RoundSession
from .multi import ShardedAggregator, ShardedRoundSession, sharded_aggregator
from .fpf import FPFTracker

__all__ = [
    "FedAvgLibraryError",
    "library_path",
    "DeviceAggregator",
    "FedAvgAggregateMixin",
    "aggregate",
    "client_arena",
    "client_distances",
    "estimate_delta",
    "client_sqdist",
    "reduce_with_sqdist",
    "default_aggregator",
    "install",
    "sample_weights",
    "KeyTable",
    "ShapeMismatchError",
    "result_dtype",
    "ALIGN_ELEMS",
    "reduce_packed",
    "reduce_tensors",
    "weights_tensor",
    "RoundSession",
    "ShardedAggregator",
    "ShardedRoundSession",
    "sharded_aggregator",
    "FPFTracker",
]
