"""A stand-in for the reference's round loop, for the zero-edit streaming tests.

The reference modules cannot travel (and FedML is absent), so this module
holds the two classes ``mfl_amd.install`` touches, shaped like the
reference's: ``Client`` (client.py: ``update_local_dataset`` :27,
``get_sample_number`` :34, ``train`` :38 returning ``(state_dict, loss, beta,
rho, acc, cycles)`` with Nones for a diverged client, :71-73) and
``FedAvgTrainer`` (``client_list`` :88, ``train`` :95 whose client loop
follows :172-219: retry until the :190 validity test passes, append
``(client.get_sample_number(), copy.deepcopy(w))`` at :199, ``w_glob =
self.aggregate(w_locals)`` at :217, ``load_state_dict`` at :219).
``install(FedAvgTrainer)`` finds ``Client`` in this module's globals, as it
finds ``client.Client`` in ``fedavg_trainer``'s.

A round is a list of client specs ``(sample_num, [attempt, ...])``; an
attempt is a state_dict (a valid result, cloned as ``net.cpu().state_dict()``
would hand out fresh tensors) or None (a diverged run: Nones, retried).
"""
from __future__ import annotations

import copy
import time
from collections import OrderedDict


class Client:
    def __init__(self, client_idx):
        self.client_idx = client_idx
        self.local_sample_number = 0
        self._attempt = None
        self.train_delay_s = 0.0

    def update_local_dataset(self, client_idx, attempt, local_sample_number):  # client.py:27
        self.client_idx = client_idx
        self._attempt = attempt
        self.local_sample_number = local_sample_number

    def get_sample_number(self):  # client.py:34
        return self.local_sample_number

    def train(self, net, local_iteration):  # client.py:38
        if self.train_delay_s:
            time.sleep(self.train_delay_s)  # the client's local training
        if self._attempt is None:  # diverged (client.py:71-73)
            return OrderedDict(), None, None, None, None, None
        if callable(self._attempt):  # a result computed from the round's global model
            return self._attempt(net)
        w = OrderedDict((k, v.clone()) for k, v in self._attempt.items())  # net.cpu().state_dict(): fresh tensors
        return w, 0.25, 0.5, 0.75, 0.9, 100.0


class FedAvgTrainer:
    client_cls = Client

    def __init__(self, model_state, rounds, n_clients=None, train_delay_s=0.0, after_append=None,
                 before_append=None, after_aggregate=None):
        self.model_global = _Model(model_state)
        self.rounds = rounds
        n = n_clients or max((len(r) for r in rounds), default=1)
        self.client_list = [self.client_cls(i) for i in range(n)]  # fedavg_trainer.py:88
        for c in self.client_list:
            c.train_delay_s = train_delay_s
        self.after_append = after_append  # test hook: (round, w_locals) -> None, e.g. a mutation
        self.before_append = before_append  # test hook: (round, client, w) -> None, between :190 and :199
        # test hook: (round, w_locals, w_glob, train results) -> None after :219, where :289-305 run
        self.after_aggregate = after_aggregate
        self.results = []
        self.timings = []

    def aggregate(self, w_locals):  # fedavg_trainer.py:441 (replaced by mfl_amd.install)
        raise AssertionError("the reference aggregate is not part of this harness")

    def train(self):  # fedavg_trainer.py:95
        for r, specs in enumerate(self.rounds):
            w_locals, trained = [], []
            t_last = time.perf_counter()
            for idx, (n, attempts) in enumerate(specs):  # :172
                client = self.client_list[idx]
                tries = iter(attempts)
                while True:  # :181-195
                    client.update_local_dataset(idx, next(tries), n)
                    w, loss, beta, rho, acc, cyc = client.train(net=self.model_global, local_iteration=1)  # :189
                    if loss is not None and beta is not None and rho is not None and acc is not None:  # :190
                        break
                trained.append((loss, beta, rho))
                if self.before_append is not None:
                    self.before_append(r, idx, w)
                t_last = time.perf_counter()
                w_locals.append((client.get_sample_number(), copy.deepcopy(w)))  # :199
            if self.after_append is not None:
                self.after_append(r, w_locals)
            t0 = time.perf_counter()
            w_glob = self.aggregate(w_locals)  # :217
            t1 = time.perf_counter()
            self.model_global.load_state_dict(w_glob)  # :219
            if self.after_aggregate is not None:
                self.after_aggregate(r, w_locals, w_glob, trained)
            self.results.append(OrderedDict((k, v.clone()) for k, v in w_glob.items()))
            self.timings.append({"aggregate_ms": (t1 - t0) * 1e3, "last_train_to_model_ms": (t1 - t_last) * 1e3})


class _Model:
    def __init__(self, state):
        self._state = OrderedDict((k, v.clone()) for k, v in state.items())

    def state_dict(self):
        return self._state

    def load_state_dict(self, sd):  # copy_ casts into each buffer's dtype, as nn.Module does
        for k, v in self._state.items():
            v.copy_(sd[k])

    def cpu(self):
        return self


def fresh_classes():
    """New (FedAvgTrainer, Client) subclasses, so that each test installs the
    drop-in on its own classes (install patches classes in place)."""

    class TestClient(Client):
        pass

    class TestTrainer(FedAvgTrainer):
        client_cls = TestClient

    return TestTrainer, TestClient


def rounds_from_cases(cases, n_rounds=1):
    """Golden cases [(meta, w_locals, expected)] -> harness rounds: round r
    replays case r % len(cases); every client valid at its first attempt."""
    rounds = []
    for r in range(n_rounds):
        _, w_locals, _ = cases[r % len(cases)]
        rounds.append([(n, [sd]) for n, sd in w_locals])
    return rounds
