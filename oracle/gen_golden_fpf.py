"""Golden vectors for the FPF2 bookkeeping, produced by the REFERENCE's own round loop.

Test infrastructure, run by hand in the build container only (the reference is
not present on the GPU box):

    python oracle/gen_golden_fpf.py [scenario ...]   # writes tests/golden/fpf/*.npz

The FPF2 state (``local_w_diffs``, ``A_mat``, ``G_mat``, ``local_itr_lst`` /
``LRU_itr_lst``; fedavg_trainer.py:108-119, :210, :271-278, :314-327) lives in
locals of ``FedAvgTrainer.train`` -- there is no function to call.  So this
script runs the reference ``train()`` itself (``fedavg_trainer.py:95-348``,
imported read-only, never copied) on a trainer whose data-side collaborators
are stubs: a scripted scheduler (client indexes + ``local_itr`` per round),
clients whose ``train`` returns the global model plus seeded noise, and no-op
``tx_time`` / ``local_test_on_all_clients``.  Everything between -- the
``w_locals`` loop, ``aggregate``, ``load_state_dict``, the FPF2 index and its
NaN/inf scrub, the ``local_w_diffs``/``A_mat``/``G_mat`` updates -- is the
reference's code.  The reference writes the per-round FPF2 list to its
``FPF_csv`` (:280-286); those rows are the expected outputs.

Scenarios: an MNIST-LR-shaped model (full mode, P < THRESHOLD_WEIGHT_SIZE),
a model with BatchNorm buffers (int64 ``num_batches_tracked``), and the LRU
mode (``THRESHOLD_WEIGHT_SIZE`` lowered below P, :117-118, :274, :323-325).
The round script covers a ``local_itr == 0`` round (no G/LRU record, :321),
an all-clients round (empty unselected set, :317) and an empty round, whose
zero global diff makes ``A_mat`` NaN (0/0 at :319) -- a reference quirk the
drop-in keeps.

Stubs for ``wandb``/``hwcounter`` and the temp-dir CWD come from
``gen_golden.py``.  Each ``.npz`` holds ``meta`` (JSON: scenario, rounds,
keys), ``init__<key>`` (initial global model), ``w__r<t>__i<j>__<key>``
(client ``j``'s returned state in round ``t``) and ``fpf`` (rounds x
client_num_in_total, the reference's CSV values as float64).
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile
import textwrap
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from gen_golden import REF_DATA, REF_SRC, _STUB_HWCOUNTER, _STUB_WANDB  # noqa: E402

REPO = Path(__file__).resolve().parents[1]
OUT_DIR = REPO / "tests" / "golden" / "fpf"

_CHILD = r'''
import copy, csv, glob, json, os, sys, types
import numpy as np
import torch

import fedavg_trainer as ft  # /root/reference/src/fedavg_trainer.py

out_dir = sys.argv[1]
N_TOTAL = 12
ROUNDS = [  # (client_indexes, local_itr) returned by the scheduler each round
    ([0, 3, 5], 2),
    ([1, 3], 3),
    ([2, 4, 6, 8, 10], 1),
    ([3, 5, 7], 0),             # local_itr == 0: nothing recorded (:321)
    (list(range(N_TOTAL)), 2),  # every client: empty unselected set (:317)
    ([11, 0], 4),
    ([], 1),                    # empty round: A_mat -> NaN (:319), kept as-is
    ([4, 9], 2),
]
SCENARIOS = [("lr_full", "lr", None), ("bn_full", "bn", None), ("lr_lru", "lr", 64),
             # round 5: models whose keys are not all fp32 (torch.cat's promotion
             # in :210 and :291, A_mat / the index in the promoted dtype)
             # (a bf16 model cannot run the reference's train(): :112 calls .numpy()
             # on every key, which raises TypeError for bfloat16)
             ("lr64_full", "lr64", None), ("lr16_full", "lr16", None),
             ("bnmix64_full", "bnmix64", None), ("lr64_lru", "lr64", 64)]
ONLY = set(sys.argv[2:])  # scenario names to (re)generate; all when empty


def make_model(kind):
    torch.manual_seed(1234)
    if kind == "lr":
        return torch.nn.Linear(100, 10)
    if kind == "lr64":
        return torch.nn.Linear(100, 10).double()
    if kind == "lr16":
        return torch.nn.Linear(100, 10).half()
    m = torch.nn.Sequential(torch.nn.Linear(16, 8), torch.nn.BatchNorm1d(8))
    if kind == "bnmix64":  # fp32 Linear, fp64 BatchNorm (its int64 counter stays int64)
        m[1].double()
    return m


state = {"round": -1}
record = {}


def scheduler(round_idx, time_counter):
    state["round"] = round_idx
    idx, itr = ROUNDS[round_idx]
    return list(idx), itr


class StubClient:
    def __init__(self, slot):
        self.slot, self.ds, self.n = slot, None, None

    def update_local_dataset(self, idx, train, test, n):
        self.ds, self.n = idx, n

    def get_sample_number(self):
        return self.n

    def train(self, net, local_iteration):
        r = state["round"]
        g = torch.Generator().manual_seed(1000 * r + self.ds)
        w = copy.deepcopy(net.cpu().state_dict())
        for k, v in w.items():
            if v.dtype == torch.int64:
                w[k] = v + local_iteration
            else:  # the noise in the key's own dtype (fp32 keys: unchanged from round 1)
                w[k] = v + (0.01 * (1 + self.ds) * torch.randn(v.shape, generator=g)).to(v.dtype)
        record[(r, self.slot)] = {k: v.clone() for k, v in w.items()}
        return w, 0.1 * (1 + self.ds), 0.5, 0.5, 0.5, 1


def run(name, kind, threshold):
    record.clear()
    ft.client_num_in_total = N_TOTAL
    ft.THRESHOLD_WEIGHT_SIZE = threshold if threshold is not None else 100000
    tr = object.__new__(ft.FedAvgTrainer)
    tr.device = torch.device("cpu")
    tr.args = types.SimpleNamespace(comm_round=len(ROUNDS), method="sch_random", frequency_of_the_test=10**6,
                                    lr=0.03, model=kind)
    tr.client_num, tr.class_num = N_TOTAL, 10
    tr.train_data_local_num_dict = {i: 10 + 7 * i for i in range(N_TOTAL)}
    tr.train_data_local_dict = {i: None for i in range(N_TOTAL)}
    tr.test_data_local_dict = {i: None for i in range(N_TOTAL)}
    tr.client_list = [StubClient(s) for s in range(N_TOTAL)]
    tr.invalid_datasets = {}
    tr.time_counter = ft.channel_data["Time"][0]
    tr.cycle_num = 0
    tr.scheduler = scheduler
    tr.model = lambda *a, **k: make_model(kind)
    tr.model_global = make_model(kind)
    tr.model_global.train()
    init = {k: v.clone() for k, v in tr.model_global.state_dict().items()}
    tr.local_test_on_all_clients = lambda *a, **k: (0.5, np.full(N_TOTAL, 0.5))
    tr.tx_time = lambda *a, **k: None
    for f in glob.glob(ft.FPF_csv):
        os.remove(f)
    tr.train()
    with open(ft.FPF_csv, newline="") as fh:
        rows = list(csv.reader(fh))
    os.remove(ft.FPF_csv)
    assert rows[0][0] == "time counter" and len(rows) == len(ROUNDS) + 1, rows[:2]
    fpf = np.array([[float(x) for x in row[1:]] for row in rows[1:]], dtype=np.float64)
    weight_size = sum(v.numel() for v in init.values())
    meta = {"scenario": name, "model": kind, "client_num_in_total": N_TOTAL, "comm_round": len(ROUNDS),
            "threshold": ft.THRESHOLD_WEIGHT_SIZE, "weight_size": weight_size,
            "full": weight_size < ft.THRESHOLD_WEIGHT_SIZE, "G1": ft.G1, "G2": ft.G2,
            "rounds": [{"client_indexes": idx, "local_itr": itr,
                        "sample_nums": [10 + 7 * c for c in idx]} for idx, itr in ROUNDS],
            "keys": [{"name": k, "shape": list(v.shape), "dtype": str(v.dtype).replace("torch.", "")}
                     for k, v in init.items()]}
    arrays = {"meta": np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8), "fpf": fpf}
    raw = lambda v: v.view(torch.int16).numpy() if v.dtype == torch.bfloat16 else v.numpy()  # numpy has no bf16
    for k, v in init.items():
        arrays[f"init__{k}"] = raw(v)
    for (r, j), w in record.items():
        for k, v in w.items():
            arrays[f"w__r{r}__i{j}__{k}"] = raw(v)
    np.savez_compressed(os.path.join(out_dir, name + ".npz"), **arrays)
    print(name, "P =", weight_size, "full =", meta["full"], "nonzero fpf per round:",
          [int(np.count_nonzero(r)) for r in fpf])


for name, kind, threshold in SCENARIOS:
    if not ONLY or name in ONLY:
        run(name, kind, threshold)
'''


def main() -> int:
    if not (REF_SRC / "fedavg_trainer.py").exists():
        print("reference not present; golden vectors can only be generated in the build container")
        return 1
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    with tempfile.TemporaryDirectory(prefix="fedavg_fpf_golden_") as tmp:
        tmp = Path(tmp)
        stubs = tmp / "stubs"
        stubs.mkdir()
        (stubs / "wandb.py").write_text(textwrap.dedent(_STUB_WANDB))
        (stubs / "hwcounter.py").write_text(textwrap.dedent(_STUB_HWCOUNTER))
        (tmp / "data").symlink_to(REF_DATA)
        run = tmp / "run"
        run.mkdir()
        child = tmp / "child.py"
        child.write_text(_CHILD)
        env = dict(os.environ)
        env["PYTHONPATH"] = f"{stubs}:{REF_SRC}"
        env["PYTHONDONTWRITEBYTECODE"] = "1"
        env["CUDA_VISIBLE_DEVICES"] = ""
        proc = subprocess.run([sys.executable, str(child), str(OUT_DIR), *sys.argv[1:]], cwd=run, env=env)
        return proc.returncode


if __name__ == "__main__":
    sys.exit(main())
