"""The written expectation for the driver's 1/2/4/8-GPU runs.

    python scripts/predict_scale.py [--shards gpurun_out/r06/shards] [--out profiles/r06/scale_prediction.json]

Inputs, all measured on one MI355X except the xGMI rate:
* the per-rank kernel fraction of each strong-scaled plan at N = 2/4/8
  (``bench.py --shard-of N``: rank 0's shard in its chunks, no exchange;
  profiles/r06/shards/*.json) and its per-step reduce time;
* the all-gather every rank receives: (N - 1) / N x 4 P bytes;
* the xGMI in-rate per rank, a range: LOW = one link's 153 GB/s (the task
  statement's per-link figure: a 2-GPU pair has one link; a single ring per
  step), HIGH = max(153, 0.75 x (N - 1) x 153) GB/s (every peer link busy at
  the efficiency RCCL's all-gather reaches on MI300X-class nodes);
* the share of the shorter leg the chunked pipeline hides, h = 0.75 (the
  overlap probe at the N = 8 rank shape: 56 % at 2 chunks, 77 % at 4, 87 % at
  8), plus 20 us of RCCL call latency per step.

step = max(t_reduce, t_gather) + (1 - h) * min(t_reduce, t_gather) + 20 us;
value = 4 K P + 4 P + 4 K bytes / step; step_frac_of_node_hbm = value / (N x 8 TB/s).
"""
from __future__ import annotations

import argparse
import json
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
HBM = 8000.0  # GB/s per GPU
LINK = 153.0  # GB/s per xGMI link (task statement)
HIDE = 0.75
RCCL_US = 20.0
WORKLOADS = {"target": (100, 25_000_000), "resnet18_gn": (500, 11_227_812),
             "synthetic_1000x100m": (1000, 100_000_000)}


def load_line(path: Path) -> dict:
    return json.loads(path.read_text().strip().splitlines()[-1])


def predict(shards: Path) -> dict:
    out = {"assumptions": {"xgmi_link_GBps": LINK, "in_rate_low": "one link (153 GB/s)",
                           "in_rate_high": "max(1, 0.75 x (N - 1)) links", "hidden_fraction": HIDE,
                           "rccl_latency_us_per_step": RCCL_US, "hbm_peak_GBps": HBM},
           "bar": 0.70, "workloads": {}}
    for w, (K, P) in WORKLOADS.items():
        alg = 4 * K * P + 4 * P + 4 * K
        rows = {}
        for n in (2, 4, 8):
            f = shards / f"{w}_s{n}.json"
            if not f.exists():
                continue
            d = load_line(f)
            kfrac = d["roofline"]["frac"]
            t_red = d["ms_per_step"]  # the rank's reduce step (its chunks, no exchange)
            gbytes = (n - 1) / n * 4 * P
            pred = {}
            for label, rate in (("low", LINK), ("high", max(LINK, 0.75 * (n - 1) * LINK))):
                t_g = gbytes / (rate * 1e9) * 1e3
                step = max(t_red, t_g) + (1 - HIDE) * min(t_red, t_g) + RCCL_US / 1e3
                value = alg / (step * 1e-3) / 1e9
                pred[label] = {"gather_ms": round(t_g, 4), "step_ms": round(step, 4), "value_GBps": round(value, 1),
                               "step_frac_of_node_hbm": round(value / (n * HBM), 4)}
            rows[str(n)] = {"per_rank_kernel_frac": kfrac, "per_rank_reduce_ms": t_red,
                            "chunks": d["config"]["chunks"], "gather_in_MB_per_rank": round(gbytes / 1e6, 1),
                            "bound": "exchange" if pred["low"]["gather_ms"] > t_red else "hbm",
                            "predicted": pred, "source": str(f.relative_to(ROOT)) if f.is_relative_to(ROOT) else str(f)}
        out["workloads"][w] = rows
    return out


def table(pred: dict) -> str:
    lines = ["| workload | N | per-rank kernel | reduce ms | gather in (MB) | gather ms (low / high) | step ms | value GB/s | step / node HBM |",
             "|---|---|---|---|---|---|---|---|---|"]
    for w, rows in pred["workloads"].items():
        for n, r in rows.items():
            lo, hi = r["predicted"]["low"], r["predicted"]["high"]
            lines.append(f"| {w} | {n} | {r['per_rank_kernel_frac']:.3f} | {r['per_rank_reduce_ms']:.3f} | "
                         f"{r['gather_in_MB_per_rank']:.1f} | {lo['gather_ms']:.3f} / {hi['gather_ms']:.3f} | "
                         f"{hi['step_ms']:.3f}-{lo['step_ms']:.3f} | {lo['value_GBps']:,.0f}-{hi['value_GBps']:,.0f} | "
                         f"{lo['step_frac_of_node_hbm']:.2f}-{hi['step_frac_of_node_hbm']:.2f} |")
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", default=str(ROOT / "profiles" / "r06" / "shards"))
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r06" / "scale_prediction.json"))
    args = ap.parse_args()
    pred = predict(Path(args.shards))
    Path(args.out).write_text(json.dumps(pred, indent=1) + "\n")
    print(table(pred))


if __name__ == "__main__":
    main()
