"""CPU oracle for the FPF2 bookkeeping -- TEST INFRASTRUCTURE ONLY.

Restates, in the reference's own torch fp32 expressions, the per-round FPF2
state updates of ``FedAvgTrainer.train`` (/root/reference/src/fedavg_trainer.py):

* :108-119  state: ``local_itr_lst [comm_round, N]``, ``G_mat [N]``, and either
            ``A_mat [P]`` + ``local_w_diffs [N, P]`` (P < THRESHOLD_WEIGHT_SIZE)
            or ``LRU_itr_lst [N]``
* :209-210  ``local_w_diffs[client_idx] = cat(w - last_w)`` per trained client
* :271-278  ``FPF2 = norm(local_w_diffs * A_mat, dim=1) / G_mat`` (or
            ``LRU_itr_lst / G_mat``), NaN/inf -> 0
* :314-319  unselected rows ``-= global_w_diff``; ``A_mat`` EMA
* :320-327  ``local_itr_lst`` / ``LRU_itr_lst`` record and the ``G_mat`` EMA

Constants from config.py:74-75 (G1 = G2 = 2) and :83 (THRESHOLD_WEIGHT_SIZE).
Pinned by ``tests/golden/fpf`` (the reference's own ``train()`` loop, see
``gen_golden_fpf.py``): replaying those rounds through this class reproduces
the reference's FPF CSV bit for bit (tests/test_oracle_golden.py).  Only
``tests/`` and ``__graft_entry__.smoke()`` may import this module; the
product (``mfl_amd.FPFTracker``) runs HIP kernels and never calls it.
"""
from __future__ import annotations

import numpy as np
import torch

G1 = 2  # config.py:74
G2 = 2  # config.py:75
THRESHOLD_WEIGHT_SIZE = 100000  # config.py:83


class FPFOracle:
    def __init__(self, client_num_in_total, weight_size, comm_round, threshold=THRESHOLD_WEIGHT_SIZE,
                 g1=G1, g2=G2, device="cpu"):
        """``device``: where the reference keeps the state (``self.device``);
        "cpu" for parity, a GPU only for bench.py's torch-on-GPU baseline."""
        n = int(client_num_in_total)
        self.n, self.g1, self.g2, self.device = n, g1, g2, device
        self.local_itr_lst = torch.zeros(comm_round, n).to(device)  # :109
        self.G_mat = torch.zeros(n).to(device)  # :110
        self.full = weight_size < threshold  # :113
        if self.full:
            self.A_mat = torch.ones(weight_size).to(device)  # :114
            self.local_w_diffs = torch.zeros((n, weight_size)).to(device)  # :115
        else:
            self.LRU_itr_lst = torch.zeros(n).to(device)  # :118

    def record_client(self, client_idx, w, last_w):
        """:209-210 (keys in ``last_w``'s order, like the model's state_dict)."""
        if self.full:
            self.local_w_diffs[client_idx, :] = torch.cat(
                [w[k].reshape((-1,)) - last_w[k].reshape((-1,)) for k in last_w.keys()]).to(self.device)

    def fpf_index(self) -> np.ndarray:
        """:271-278."""
        if self.full:
            fpf = torch.norm(self.local_w_diffs * self.A_mat, dim=1) / self.G_mat
        else:
            fpf = self.LRU_itr_lst / self.G_mat
        fpf = fpf.cpu().numpy()
        fpf[np.bitwise_or(np.isnan(fpf), np.isinf(fpf))] = 0
        return fpf

    def end_round(self, round_idx, client_indexes, local_itr, w_glob, last_w):
        """:314-327."""
        if self.full:
            gdiff = torch.cat([w_glob[k].reshape((-1,)) - last_w[k].reshape((-1,))
                               for k in last_w.keys()]).to(self.device)
            self.local_w_diffs[list(set(list(range(self.n))) - set(list(client_indexes))), :] -= gdiff
            self.A_mat = self.A_mat * (1 - 1 / self.g2) + gdiff / self.g2 / gdiff.mean()
        if list(client_indexes) and local_itr > 0:
            self.local_itr_lst[round_idx, list(client_indexes)] = float(local_itr)
            if not self.full:
                self.LRU_itr_lst += float(local_itr)
                self.LRU_itr_lst[list(client_indexes)] = 0
        self.G_mat = self.G_mat * (1 - 1 / self.g1) + self.local_itr_lst[round_idx, :] / self.g1
