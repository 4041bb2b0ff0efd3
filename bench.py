#!/usr/bin/env python3
"""bench.py -- learner env-steps/s of the MI355X IMPALA learner step (BASELINE.json metric).

One "step" = one full learner step (policy forward -> V-trace + loss + analytic grads ->
policy backward -> [RCCL all-reduce] -> optimizer) over one (T, B) batch of synthetic
trajectories already resident in HBM. value = T * B_per_gpu * N * K / max-over-ranks(time).

  python bench.py [--gpus N --steps K --warmup W] [--arch atari|mlp]
  N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

The roofline object is measured live: HIP events around every kernel launch of a few
profiled steps (after the timed region) give each kernel's mean duration; ALGORITHMIC work
per launch / duration vs the MI355X peak. cpu_baseline times the C
oracle (oracle/, kind "port") on rank 0 on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "learner env-steps/sec (T×B/step) at T=100 B=4096, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}  # dense peaks (no sparsity)
VT_REPLAYS = 100  # back-to-back V-trace launches per timing (the events' own overhead over 20 was ~2 %)


def kernel_work(arch, T, B, A, D=128, H=256):
    """Algorithmic work per launch for each tagged kernel site: (flops, bytes).
    The roofline bound is whichever of MFMA or HBM time at peak is larger."""
    R = (T + 1) * B
    TB = T * B
    w = {"vtrace": (0, (12 * A + 28) * TB)}
    if arch == "mlp":
        O = A + 1
        f32 = 4
        w.update({
            "mlp_fwd_l1": (2 * R * D * H, R * f32 * (D + H)), "mlp_fwd_l2": (2 * R * H * H, R * f32 * 2 * H),
            "mlp_fwd_heads": (2 * R * H * O, R * f32 * (H + O)), "mlp_wgrad_heads": (2 * R * H * O, R * f32 * (H + O)),
            "mlp_dgrad_heads": (2 * R * O * H, R * f32 * (O + 2 * H)), "mlp_wgrad_l2": (2 * R * H * H, R * f32 * 2 * H),
            "mlp_dgrad_l2": (2 * R * H * H, R * f32 * 3 * H), "mlp_wgrad_l1": (2 * R * D * H, R * f32 * (D + H)),
        })
    else:
        from freeimpala_amd.atari_shapes import atari_kernel_work
        w.update(atari_kernel_work(T, B, A))
    return w


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def cpu_baseline(arch, T, A, seconds, threads):
    """Time the C oracle (test infrastructure, kind 'port') on a bounded sample."""
    import numpy as np
    from oracle import oracle as orc
    orc.set_threads(threads)
    if arch == "mlp":
        D, H = 128, 256

        def one(Bs):
            batch = orc.synth_batch(42, T=T, B=Bs, A=A, D=D)
            p = np.random.RandomState(0).uniform(-0.05, 0.05, orc.mlp_param_count(D, H, A)).astype(np.float32)
            m = np.zeros_like(p)
            v = np.zeros_like(p)
            t0 = time.perf_counter()
            obs = batch["obs"].reshape((T + 1) * Bs, D)
            h1, h2, out = orc.mlp_forward(obs, p, H=H, A=A)
            logits = out[:, :A].reshape(T + 1, Bs, A)
            values = out[:, A].reshape(T + 1, Bs)
            vt = orc.vtrace_loss(logits[:T], batch["mu"], batch["actions"], batch["rewards"],
                                 batch["discounts"], values)
            dout = np.zeros(((T + 1) * Bs, A + 1), np.float32)
            dout[:T * Bs, :A] = vt["dlogits"].reshape(T * Bs, A)
            dout[:, A] = vt["dvalue"].reshape(-1)
            g = orc.mlp_backward(obs, p, h1, h2, dout, H=H, A=A)
            orc.clip_grad_norm(g, 40.0)
            orc.adam(p, g, m, v, 5e-4, 0.9, 0.999, 1e-8, 1)
            return time.perf_counter() - t0
        sample = "oracle MLP learner step (fwd+vtrace+bwd+adam), T=%d" % T
    else:
        def one(Bs):
            batch = orc.synth_batch(42, T=T, B=Bs, A=A, D=1, obs=False, frames=True)
            n = orc.atari_param_count(A)
            p = np.random.RandomState(0).uniform(-0.02, 0.02, n).astype(np.float32)
            m = np.zeros_like(p)
            v = np.zeros_like(p)
            t0 = time.perf_counter()
            fr = batch["frames"].reshape((T + 1) * Bs, 84, 84, 4)
            acts = orc.atari_forward(fr, p, A=A, bf16_emul=False)
            out = acts["out"]
            logits = out[:, :A].reshape(T + 1, Bs, A)
            values = out[:, A].reshape(T + 1, Bs)
            vt = orc.vtrace_loss(logits[:T], batch["mu"], batch["actions"], batch["rewards"],
                                 batch["discounts"], values)
            dout = np.zeros(((T + 1) * Bs, A + 1), np.float32)
            dout[:T * Bs, :A] = vt["dlogits"].reshape(T * Bs, A)
            dout[:, A] = vt["dvalue"].reshape(-1)
            g = orc.atari_backward(fr, p, acts, dout, A=A, bf16_emul=False)
            orc.clip_grad_norm(g, 40.0)
            orc.adam(p, g, m, v, 5e-4, 0.9, 0.999, 1e-8, 1)
            return time.perf_counter() - t0
        sample = "oracle Atari-net learner step (fwd+vtrace+bwd+adam, fp32/fp64), T=%d" % T
    Bs = 1
    t = one(Bs)
    # scale the sample so one measured step takes ~seconds/2, then time 2 of them
    target = max(1.0, seconds / 2.0)
    Bs = max(1, min(4096, int(Bs * target / max(t, 1e-3))))
    ts = [one(Bs) for _ in range(2)]
    step = min(ts)
    # V-trace + loss + grads alone at the full config size
    case = orc.synth_batch(7, T=T, B=4096, A=A, D=1, obs=False)
    rs = np.random.RandomState(1)
    pi = rs.randn(T, 4096, A).astype(np.float32)
    val = rs.randn(T + 1, 4096).astype(np.float32)
    t0 = time.perf_counter()
    orc.vtrace_loss(pi, case["mu"], case["actions"], case["rewards"], case["discounts"], val)
    tv = time.perf_counter() - t0
    return {
        "value": T * Bs / step, "unit": "env-steps/s", "cores": threads, "kind": "port",
        "sample": f"{sample}, B={Bs} per step (min of 2 steps, {step:.2f} s each)",
        "vtrace_only": {"value": T * 4096 / tv, "unit": "env-steps/s",
                        "sample": f"oracle V-trace+loss+grads at T={T} B=4096 A={A}"},
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--arch", default=os.environ.get("FI_BENCH_ARCH", "atari"), choices=["atari", "mlp"])
    ap.add_argument("--seq-len", type=int, default=100)
    ap.add_argument("--batch", type=int, default=4096, help="per-GPU batch (weak scaling)")
    ap.add_argument("--num-actions", type=int, default=18)
    ap.add_argument("--profile-steps", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    N = max(ws, 1)
    # the learner library first: it then binds the image's ROCm 7.2 runtime, hipBLASLt and RCCL
    # (what it is built against, and what the tests and smoke() load); imported first, torch's
    # bundled ROCm 7.0 copies would take those sonames. torch is only the gloo launcher here
    # and never touches the GPU.
    if os.environ.get("FI_BENCH_TORCH_FIRST"):  # A/B only: torch's bundled ROCm libraries
        import torch  # noqa: F401
    from freeimpala_amd import _abi
    _abi.lib()
    import torch  # noqa: F401,F811
    import torch.distributed as dist
    if ws > 1:
        dist.init_process_group("gloo", rank=rank, world_size=ws)

    from freeimpala_amd.launch import broadcast_bytes, max_over_ranks, shard_columns
    from freeimpala_amd.learner import DeviceLearner

    T, B, A = args.seq_len, args.batch, args.num_actions
    # rehearsal knobs for a one-GPU box (never set by the driver): FI_BENCH_DEVICE pins every
    # rank to one device, FI_BENCH_NO_COMM skips the RCCL communicator (RCCL refuses two ranks
    # on one device), so the launcher path (torchrun env, gloo, shards, barrier, max) runs
    device = int(os.environ.get("FI_BENCH_DEVICE", local))
    L = DeviceLearner(args.arch, seq_len=T, batch=B, num_actions=A, device=device,
                      optimizer="adam", publish="bf16" if args.arch == "atari" else "fp32")
    b_off, _ = shard_columns(rank, N, B)
    L.synth(seed=42, b_global=B * N, b_offset=b_off)
    if ws > 1 and not os.environ.get("FI_BENCH_NO_COMM"):  # RCCL communicator for the in-step gradient all-reduce (uid via gloo)
        uid = broadcast_bytes(DeviceLearner.comm_unique_id() if rank == 0 else b"", 0)
        L.attach_comm(uid, rank, ws)

    def barrier():
        L.sync()
        if ws > 1:
            dist.barrier()

    for _ in range(args.warmup):
        L.step_resident(stats=False)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        L.step_resident(stats=False)
    L.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    if ws > 1:
        elapsed = max_over_ranks(elapsed)
    ms_per_step = 1000.0 * elapsed / args.steps
    value = T * B * N * args.steps / elapsed

    # ---- live per-kernel timing (HIP events on the learner stream) for the roofline
    L.set_profiling(True)
    for _ in range(args.profile_steps):
        L.step_resident(stats=False)
    kt = kernel_times(L)
    phases = L.phase_times()
    L.set_profiling(False)
    vt_replay_ms = L.replay_vtrace(VT_REPLAYS)  # the scan kernel alone, back-to-back (see roof_vtrace)
    st = L.step_resident(stats=True)

    work = kernel_work(args.arch, T, B, A)
    # HBM bytes per launch from the committed rocprofv3 PMC passes (scripts/pmc_pass.sh,
    # corrected as MI355X_MICROARCH.md prescribes); only valid for the same T/B/A config
    traffic = {}
    tpath = os.path.join(ROOT, "profiles", f"r01_pmc_traffic_{args.arch}.json")
    if os.path.exists(tpath) and (T, B, A) == (100, 4096, 18):
        with open(tpath) as fh:
            traffic = {k: v["hbm_bytes_per_launch"] for k, v in json.load(fh).items() if not k.startswith("_")}
    # MFMA utilisation and effective clock per kernel from the committed counter pass
    # (scripts/pmc_mfma.sh), same config only
    mfma = {}
    mpath = os.path.join(ROOT, "profiles", f"r01_pmc_mfma_{args.arch}.json")
    if os.path.exists(mpath) and (T, B, A) == (100, 4096, 18):
        with open(mpath) as fh:
            mfma = {k: v for k, v in json.load(fh).items() if not k.startswith("_")}
    per_step = {k: v["ms"] * v["count"] / max(1, args.profile_steps) for k, v in kt.items()}
    dominant = max(per_step, key=per_step.get) if per_step else None
    dtype = "bf16" if args.arch == "atari" else "fp32"

    def roof(name, ms=None):
        if name not in kt or name not in work:
            return None
        flops, nbytes = work[name]
        ms = kt[name]["ms"] if ms is None else ms
        tr = traffic.get(name)
        peak_f = MFMA_PEAK_TFLOPS[dtype] * 1e12
        t_mfma, t_hbm = flops / peak_f, nbytes / (HBM_PEAK_GBS * 1e9)
        common = {"kernel": name, "traffic": tr, "launch_ms": round(ms, 5),
                  "mfma_util_pmc": mfma.get(name, {}).get("mfma_util"),
                  "clock_mhz_pmc": mfma.get(name, {}).get("clock_mhz"),
                  "algorithmic_flops": flops, "algorithmic_bytes": nbytes,
                  "time_at_peak_ms": {"mfma": round(t_mfma * 1e3, 4), "hbm": round(t_hbm * 1e3, 4)}}
        if t_hbm >= t_mfma:
            ach = nbytes / (ms * 1e-3) / 1e9
            return dict(common, bound="hbm", achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                        frac=round(ach / HBM_PEAK_GBS, 4))
        ach = flops / (ms * 1e-3) / 1e12
        return dict(common, bound="mfma", achieved=round(ach, 2), peak=MFMA_PEAK_TFLOPS[dtype],
                    unit="TFLOP/s", frac=round(ach / MFMA_PEAK_TFLOPS[dtype], 4))

    result = {
        "metric": METRIC, "value": round(value, 1), "unit": "env-steps/s", "n_gpus": N,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": dtype,
        "data": "synthetic (Philox4x32-10 on device, resident in HBM; random-init Glorot params)",
        "config": {
            "workload": ("config#3 Atari-shaped conv policy 84x84x4, bf16 MFMA GEMMs + fp32 V-trace"
                         if args.arch == "atari" else
                         "MLP policy 128-256-256 fp32 (config#2 network) at the metric's T/B"),
            "T": T, "B_per_gpu": B, "A": A, "global_batch": B * N, "seq_len": T,
            "parallelism": f"dp{N}", "optimizer": "adam", "policy": args.arch,
        },
        "roofline": roof(dominant) if dominant else None,
        # V-trace scan: ~20 us, so per-launch event brackets inside the step carry the dispatch
        # latency; the burst of VT_REPLAYS back-to-back launches on the same resident tensors is the
        # kernel's duration (agrees with rocprofv3's kernel-trace average)
        "roofline_vtrace": dict(roof("vtrace", vt_replay_ms) or {},
                                method=f"HIP events around {VT_REPLAYS} back-to-back launches",
                                in_step_event_ms=round(kt["vtrace"]["ms"], 5) if "vtrace" in kt else None),
        "kernel_ms_per_step": {k: round(v, 4) for k, v in sorted(per_step.items(), key=lambda x: -x[1])},
        "phase_ms": {k: round(v, 4) for k, v in phases.items() if k != "steps"},
        "final_loss": st["total_loss"], "grad_norm": st["grad_norm"],
    }
    if rank == 0 and N == 1 and not args.no_cpu_baseline:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
        threads = min(threads, 16)
        try:
            result["cpu_baseline"] = cpu_baseline(args.arch, T, A, args.cpu_seconds, threads)
            result["speedup_vs_cpu"] = round(value / result["cpu_baseline"]["value"], 1)
        except Exception as e:  # the baseline is reported, never blocks the GPU number
            result["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    L.close()
    if ws > 1:
        dist.destroy_process_group()


def kernel_times(L):
    import ctypes as C
    from freeimpala_amd._abi import lib
    buf = C.create_string_buffer(8192)
    ms = (C.c_float * 128)()
    cnt = (C.c_int * 128)()
    n = lib().fi_learner_kernel_times(L._h, buf, 8192, ms, cnt, 128)
    names = buf.value.decode().split("\n")[:n]
    return {names[i]: {"ms": ms[i], "count": cnt[i]} for i in range(n)}


if __name__ == "__main__":
    main()
