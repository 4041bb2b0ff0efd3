#!/usr/bin/env python3
"""FarmerLstm train-step throughput (the reference's own benchmark metric: samples/second =
batch_size / mean step time, scripts/gpu_benchmark.py:264-277) on one MI355X, with the
reference's CPU execution stack (torch CPU, oracle/farmer_torch.py) timed beside it.

  python scripts/farmer_bench.py [--configs 32x10,512x100] [--steps 20 --warmup 5]

Inputs are resident in HBM before the timed region (the reference regenerates them per run on
its device; on the host that is a separate copy). One JSON line per config.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="32x10,512x100", help="BxT list (gpu_benchmark defaults 32x10)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--loss", default="mse")
    ap.add_argument("--optimizer", default="adam")
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()
    from freeimpala_amd import farmer, hip
    from oracle import farmer_oracle as fo
    for spec in args.configs.split(","):
        B, T = (int(v) for v in spec.split("x"))
        p0 = fo.gen_params(1)
        z, x, y = fo.gen_inputs(2, B, T)
        M = farmer.FarmerLstmModel(B, T, args.loss, args.optimizer, 1e-3, params=p0)
        M.upload_inputs(z, x, y)
        for _ in range(args.warmup):
            M.train_step_resident(stats=False)
        hip.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            M.train_step_resident(stats=False)
        hip.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        st_loss = M.train_step_resident(stats=True)  # + the device time of one step (HIP events)
        fwd_ms, bwd_ms = M.recurrence_ms(5)
        # recurrence rooflines: fp32 VALU (packed FMAs; 157.3 TF/s dense fp32 = the MFMA fp32 rate);
        # algorithmic work = the h W_hh^T / dgates W_hh matvecs, 2 B T H 4H flops per kernel
        fl = 2.0 * B * T * 128 * 512
        roof = {}
        for nm, ms in (("lstm_fwd", fwd_ms), ("lstm_bwd", bwd_ms)):
            ach = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
            roof[nm] = {"launch_ms": round(ms, 5), "bound": "fp32", "algorithmic_flops": fl,
                        "achieved": round(ach, 2), "peak": 157.3, "unit": "TFLOP/s", "frac": round(ach / 157.3, 4)}
        res = {"metric": "FarmerLstm train step samples/s (gpu_benchmark.py throughput)", "B": B, "T": T,
               "loss": args.loss, "optimizer": args.optimizer, "value": round(B / dt, 1), "unit": "samples/s",
               "ms_per_step": round(dt * 1e3, 4), "device_ms_one_step": round(M.last_step_ms, 4),
               "steps": args.steps, "dtype": "fp32",
               "final_loss": st_loss, "data": "synthetic N(0,1) (numpy seed 2), resident in HBM",
               "roofline": roof}
        M.close()
        if not args.no_cpu:
            import torch
            from oracle.farmer_torch import TorchFarmer
            threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
            torch.set_num_threads(threads)
            tf = TorchFarmer(p0, args.loss, args.optimizer, 1e-3)
            zt, xt, yt = (torch.from_numpy(a) for a in (z, x, y))
            tf.step(zt, xt, yt)
            t0 = time.perf_counter()
            for _ in range(args.cpu_steps):
                tf.step(zt, xt, yt)
            cdt = (time.perf_counter() - t0) / args.cpu_steps
            res["cpu_baseline"] = {"value": round(B / cdt, 1), "unit": "samples/s", "ms_per_step": round(cdt * 1e3, 2),
                                   "cores": threads, "kind": "port",
                                   "sample": f"torch-CPU FarmerLstm train step (the reference's stack), "
                                             f"{args.cpu_steps} steps at B={B} T={T}"}
            res["speedup_vs_cpu"] = round(res["value"] / res["cpu_baseline"]["value"], 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
