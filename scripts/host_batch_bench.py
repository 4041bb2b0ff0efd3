"""PCIe-inclusive learner rate: the step fed from host SharedBuffer entries (what
Learner::trainModel hands over after SharedBuffer::readBatch, data_structures.h:267-300)
against the step on a batch already resident in HBM (bench.py's `value`).

usage: python scripts/host_batch_bench.py [--T 100] [--B 4096] [--steps 8]
MLP policy only: entries follow the 1 KiB record schema, T+1 records
each; the Atari config is device-synthetic (28 KB frames do not fit a record, and
fi_learner_step refuses it). Prints one JSON line:
  resident    env-steps/s of fi_learner_step_resident
  host_serial        fi_learner_step: pinned staging copy + one H2D + ingest + step, returns
                     when done
  host_async         fi_learner_step_async x steps, then fi_learner_wait: the staging copy and
                     H2D of batch k+1 (copy stream, second device slot) overlap the device
                     step of batch k
  host_staged_h2d    fi_learner_acquire_staging + fi_learner_step_staged_async on buffers
                     the caller filled beforehand (its readBatchInto copy not timed): H2D +
                     step alone, the PCIe bound
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=100)
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=8)
    args = ap.parse_args()
    from freeimpala_amd.learner import DeviceLearner, HostBatch, pack_records
    T, B, A = args.T, args.B, 18
    L = DeviceLearner("mlp", seq_len=T, batch=B, num_actions=A, optimizer="adam")
    L.synth(seed=42)
    D = 128
    obs = L.tensor("obs", shape=(T + 1, B, D))
    mu = L.tensor("mu", shape=(T, B, A))
    act = L.tensor("actions", np.int32, (T, B))
    rew = L.tensor("rewards", shape=(T, B))
    disc = L.tensor("discounts", shape=(T, B))
    t0 = time.perf_counter()
    entries = HostBatch(pack_records(obs, mu, act, rew, disc, entry_size=T + 1))
    pack_s = time.perf_counter() - t0
    eb = entries.entry_bytes

    def timed(fn, n):
        fn()
        L.sync()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        L.sync()
        return (time.perf_counter() - t) / n

    res = timed(lambda: L.step_resident(stats=False), args.steps)
    # serial: fi_learner_step returns when the step is done (copy, H2D, step back to back)
    ser = timed(lambda: L.step(entries, stats=False), args.steps)
    # pipelined: fi_learner_step_async; copy + H2D of batch k+1 beside the step of batch k
    L.step_async(entries)
    L.wait()
    t = time.perf_counter()
    for _ in range(args.steps):
        c = time.perf_counter()
        L.step_async(entries)
        if os.environ.get("FI_STAGE_TIMING"):
            print(f"[async call] {1e3 * (time.perf_counter() - c):.3f} ms", file=sys.stderr, flush=True)
    L.wait()
    asy = (time.perf_counter() - t) / args.steps
    # staged: the caller's readBatchInto fills the acquired pinned buffer (done once here:
    # the loop then times H2D + step alone, the PCIe bound of the staged path)
    stride = L.entry_bytes
    src = np.stack([np.frombuffer(b, np.uint8)[:stride] for b in entries.bufs])
    for _ in range(2):
        np.copyto(L.acquire_staging(), src)
        L.step_staged_async()
    L.wait()
    t = time.perf_counter()
    for _ in range(args.steps):
        L.acquire_staging()
        L.step_staged_async()
    L.wait()
    stg = (time.perf_counter() - t) / args.steps
    mb = B * eb / 1e6
    out = {
        "arch": "mlp", "T": T, "B": B, "entry_bytes": eb, "batch_mb": round(mb, 1),
        "resident": {"ms_per_step": round(1e3 * res, 3), "env_steps_per_s": round(T * B / res, 1)},
        "host_serial": {"ms_per_step": round(1e3 * ser, 3), "env_steps_per_s": round(T * B / ser, 1)},
        "host_async": {"ms_per_step": round(1e3 * asy, 3), "env_steps_per_s": round(T * B / asy, 1),
                       "batch_gb_s": round(mb / 1e3 / asy, 1)},
        "host_staged_h2d": {"ms_per_step": round(1e3 * stg, 3), "env_steps_per_s": round(T * B / stg, 1),
                            "batch_gb_s": round(mb / 1e3 / stg, 1)},
        "pack_records_s": round(pack_s, 2),
    }
    print(json.dumps(out), flush=True)
    L.close()


if __name__ == "__main__":
    main()
