#!/usr/bin/env python3
"""bench.py -- learner env-steps/s of the MI355X IMPALA learner step (BASELINE.json metric).

One "step" = one full learner step (policy forward -> V-trace + loss + analytic grads ->
policy backward -> [RCCL all-reduce] -> optimizer) over one (T, B) batch of synthetic
trajectories already resident in HBM. value = T * B_per_gpu * N * K / max-over-ranks(time).

  python bench.py [--gpus N --steps K --warmup W] [--arch atari|mlp]
  N > 1 either form: `python bench.py --gpus N` starts the N ranks itself (a child
  `python -m torch.distributed.run --nproc-per-node N bench.py ...`, launched before anything
  touches the GPU; rank 0's line is relayed, the child's exit code returned), or
  `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...` directly.
  --gpus N with fewer than N visible devices, or disagreeing with a launcher's WORLD_SIZE, exits 2.

The roofline object is measured live: HIP events around every kernel launch of a few
profiled steps (after the timed region) give each kernel's mean duration; ALGORITHMIC work
per launch / duration vs the MI355X peak. cpu_baseline times the
torch-CPU port of the step under oracle/ (kind "port") on rank 0: whole T x 4096 steps (the
Atari step takes ~50 s on 16 cores and ~120 GB of host memory; with less headroom, or
--cpu-sample, a bounded sample extrapolated to B=4096).
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
VT_COLD_SETS = 6  # disjoint tensor sets the cold V-trace replay rotates over (6 x 100 MB > 256 MB MALL)


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
            # fused heads backward: reads h2 and the upstream gradient once, writes dz2
            "mlp_heads_bwd": (4 * R * H * O, R * f32 * (2 * H + O)),
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


def host_cpu_info():
    """What the CPU baseline ran on: the machine's CPUs, this process's share, the model."""
    model = None
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count()
    return {"nproc": os.cpu_count(), "affinity_cpus": share, "cpu_model": model,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def host_mem_headroom_gb():
    """Host memory this process may still take: MemAvailable, capped by the cgroup's limit
    (a gpurun box caps one command at ~270 GiB of a much larger host)."""
    avail = None
    try:
        with open("/proc/meminfo") as fh:
            for line in fh:
                if line.startswith("MemAvailable:"):
                    avail = int(line.split()[1]) * 1024
    except OSError:
        pass
    try:
        with open("/sys/fs/cgroup/memory.max") as fh:
            lim = fh.read().strip()
        with open("/sys/fs/cgroup/memory.current") as fh:
            cur = int(fh.read().strip())
        if lim != "max":
            room = int(lim) - cur
            avail = room if avail is None else min(avail, room)
    except (OSError, ValueError):
        pass
    return None if avail is None else avail / 2**30


CPU_FULL_GB = 200  # the whole B=4096 Atari CPU step peaks at ~118 GB RSS (measured on a pool box)


def full_cpu_step(arch, batch, cpu_full, cpu_sample, room_gb):
    """(run one whole T x 4096 Atari CPU step?, why not). --cpu-full forces it; otherwise it
    runs at the metric's B = 4096 when the host has CPU_FULL_GB of headroom, unless
    --cpu-sample asks for the bounded, extrapolated sample. MLP steps always run whole."""
    if arch != "atari":
        return False, None
    if cpu_full:
        return True, None
    if cpu_sample:
        return False, "--cpu-sample"
    if batch != 4096:
        return False, f"B={batch}: the full step is timed at the metric's B=4096 only"
    if room_gb is None or room_gb < CPU_FULL_GB:
        return False, f"host memory headroom {room_gb and round(room_gb, 1)} GB < {CPU_FULL_GB} GB"
    return True, None


def cpu_baseline(arch, T, A, seconds, threads, full=False):
    """Time a CPU learner step on rank 0 (test infrastructure under oracle/, kind 'port'):
    the torch-CPU port of the step (oracle/torch_learner.py: oneDNN/MKL fp32 convolutions and
    GEMMs, autograd, the same V-trace/loss/clip/Adam as the C oracle; gradient-equal to it,
    tests/test_torch_baseline.py). MLP: whole T x 4096 steps. Atari: one whole T x 4096 step
    when `full` (bench.py's default when the host has the memory for it), else a bounded sample
    extrapolated flat in B. The C oracle's own V-trace + loss at the full T x 4096 is reported
    beside it."""
    import numpy as np
    import torch
    from oracle import oracle as orc
    from oracle.torch_learner import TorchLearner
    orc.set_threads(threads)
    torch.set_num_threads(threads)
    D, H = 128, 256
    n = orc.mlp_param_count(D, H, A) if arch == "mlp" else orc.atari_param_count(A)
    p0 = np.random.RandomState(0).uniform(-0.02, 0.02, n).astype(np.float32)
    batches = {}

    def one(Bs):
        if Bs not in batches:
            batches[Bs] = orc.synth_batch(42, T=T, B=Bs, A=A, D=D, obs=arch == "mlp",
                                          frames=arch == "atari")
        tl = TorchLearner(arch, p0, A=A, D=D, H=H)
        t0 = time.perf_counter()
        tl.step(batches[Bs])
        return time.perf_counter() - t0

    if arch == "mlp":
        # config #2 at B=512 and the metric's B=4096, in full (no extrapolation)
        per_b = {}
        for Bs in (512, 4096):
            per_b[Bs] = min(one(Bs) for _ in range(2))
        Bs, step = 4096, per_b[4096]
        sample = (f"torch-CPU port of the MLP learner step (fwd+vtrace+bwd+clip+adam, fp32), "
                  f"T={T}, full B=4096 (min of 2 steps, {per_b[4096]:.2f} s; B=512: {per_b[512]:.3f} s "
                  f"= {T * 512 / per_b[512]:.0f} env-steps/s)")
        extrap = False
    elif full:  # one whole T x 4096 step (~50 s on 16 cores, ~120 GB of host memory)
        import resource
        Bs = 4096
        step = one(Bs)
        rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2**20
        sample = (f"torch-CPU port of the Atari-net learner step (fwd+vtrace+bwd+clip+adam, fp32), "
                  f"T={T}, the full B=4096 (one step, {step:.1f} s, peak RSS {rss:.0f} GB)")
        extrap = False
    else:
        t = one(2)
        target = max(1.0, seconds / 3.0)
        Bs = max(2, min(4096, int(2 * target / max(t, 1e-3))))
        step = min(one(Bs) for _ in range(2))
        sample = (f"torch-CPU port of the Atari-net learner step (fwd+vtrace+bwd+clip+adam, fp32), "
                  f"T={T}, B={Bs} per step (min of 2 steps, {step:.2f} s each); EXTRAPOLATED to "
                  f"B=4096 as env-steps/s flat in B (the full B=4096 step needs {CPU_FULL_GB} GB of "
                  f"host memory headroom; bench.py --cpu-full forces it)")
        extrap = Bs < 4096
    # V-trace + loss + grads alone at the full config size (the C oracle)
    case = orc.synth_batch(7, T=T, B=4096, A=A, D=1, obs=False)
    rs = np.random.RandomState(1)
    pi = rs.randn(T, 4096, A).astype(np.float32)
    val = rs.randn(T + 1, 4096).astype(np.float32)
    t0 = time.perf_counter()
    orc.vtrace_loss(pi, case["mu"], case["actions"], case["rewards"], case["discounts"], val)
    tv = time.perf_counter() - t0
    return {
        "value": T * Bs / step, "unit": "env-steps/s", "cores": threads, "kind": "port",
        "sample": sample, "extrapolated": extrap, "host": host_cpu_info(),
        "vtrace_only": {"value": T * 4096 / tv, "unit": "env-steps/s",
                        "sample": f"C oracle V-trace+loss+grads at T={T} B=4096 A={A} ({threads} OpenMP threads)"},
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
    ap.add_argument("--sustain-seconds", type=float, default=10.0,
                    help="after the timed loop, run the step this long more and report the sustained rate")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-full", action="store_true",
                    help="time one whole T x 4096 Atari CPU step for cpu_baseline whatever the memory headroom")
    ap.add_argument("--cpu-sample", action="store_true",
                    help="Atari cpu_baseline from a bounded sample extrapolated to B=4096 (the default is "
                         f"one whole step when {CPU_FULL_GB} GB of host memory are free)")
    args = ap.parse_args()

    # --gpus N without a launcher: start the N ranks as a child launcher process before this
    # process touches the GPU (device counting through torch does not initialise it)
    import socket
    import subprocess
    from freeimpala_amd.launch import LaunchError, bench_launch_plan

    def visible_devices():
        import torch
        return torch.cuda.device_count()

    def free_port():
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            return sk.getsockname()[1]

    try:
        cmd = bench_launch_plan(args.gpus, os.environ, sys.argv[1:], os.path.abspath(__file__),
                                sys.executable, visible_devices, free_port())
    except LaunchError as e:
        print(f"bench.py: {e}", file=sys.stderr, flush=True)
        sys.exit(2)
    if cmd is not None:
        print(f"bench.py: starting {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
        sys.exit(subprocess.run(cmd).returncode)

    ws, rank, local = dist_env()
    N = max(ws, 1)
    # the learner library first: it then binds the image's ROCm 7.2 runtime and RCCL
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

    from freeimpala_amd.launch import (broadcast_bytes, data_parallel_fields, gather_objects, max_over_ranks,
                                       shard_columns, timed_steps)
    from freeimpala_amd.learner import DeviceLearner
    from freeimpala_amd.roofline import step_roofline

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
    own, elapsed = timed_steps(lambda: L.step_resident(stats=False), L.sync, barrier, args.steps)
    own_ms_per_step = 1000.0 * own / args.steps  # this rank's own clock: drained, before the closing barrier
    if ws > 1:
        elapsed = max_over_ranks(elapsed)
    ms_per_step = 1000.0 * elapsed / args.steps
    value = T * B * N * args.steps / elapsed

    # ---- sustained rate: the same step for --sustain-seconds more (untimed for `value`): the
    # power-limited clock's steady state beside the K-step burst, and GPU activity long enough
    # for a coarse utilisation sampler to see. Every rank runs the same step count (from the
    # max-over-ranks time), so the in-step all-reduces pair up.
    sustained = None
    if args.sustain_seconds > 0:
        n_sus = max(1, int(args.sustain_seconds * 1000.0 / ms_per_step))
        s_own, s_el = timed_steps(lambda: L.step_resident(stats=False), L.sync, barrier, n_sus)
        if ws > 1:
            s_el = max_over_ranks(s_el)
        sustained = {"steps": n_sus, "ms_per_step": round(1000.0 * s_el / n_sus, 4),
                     "value": round(T * B * N * n_sus / s_el, 1),
                     "note": "the same step after the timed loop, run for ~--sustain-seconds; not `value`"}

    # ---- live per-kernel timing (HIP events on the learner stream) for the roofline
    L.set_profiling(True)
    for _ in range(args.profile_steps):
        L.step_resident(stats=False)
    kt = kernel_times(L)
    phases = L.phase_times()
    L.set_profiling(False)
    # the scan kernel alone, back-to-back: cold = rotating over disjoint tensor sets larger than
    # the Infinity Cache (what the kernel gets from HBM), warm = the same resident tensors again
    vt_cold_ms = L.replay_vtrace(VT_REPLAYS, sets=VT_COLD_SETS)
    vt_warm_ms = L.replay_vtrace(VT_REPLAYS, sets=1)
    st = L.step_resident(stats=True)

    # N > 1: every rank's own ms/step and exposed all-reduce wait, the bytes all-reduced per step
    dp = None
    if ws > 1:
        comm = L.comm_info()
        dp = data_parallel_fields(gather_objects({"ms_per_step": own_ms_per_step,
                                                  "allreduce_ms": phases.get("allreduce", 0.0)}),
                                  grad_bytes=4 * L.param_count,
                                  buckets=comm["buckets_last_step"] if comm["nranks"] > 1 else None)
        if os.environ.get("FI_BENCH_NO_COMM"):
            dp["note"] = "FI_BENCH_NO_COMM rehearsal: no communicator, nothing was all-reduced"

    work = kernel_work(args.arch, T, B, A)
    # Counter fields from the committed rocprofv3 PMC summaries (scripts/pmc_pass.sh: HBM bytes
    # per launch, corrected as MI355X_MICROARCH.md prescribes; scripts/pmc_mfma.sh: MFMA busy
    # and clock), ONLY when a summary is stamped with the source hash of the tree this bench
    # runs from (freeimpala_amd/build_info.py) and the same T/B/A: counters of another build
    # are refused and the fields stay null (counters_build says which).
    traffic, mfma, counters_build = load_counters(args.arch, (T, B, A))
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
        "sustained": sustained,
        "roofline": roof(dominant) if dominant else None,
        # V-trace scan: ~20 us, so per-launch event brackets inside the step carry the dispatch
        # latency; the burst of VT_REPLAYS back-to-back launches on the same resident tensors is the
        # kernel's duration (agrees with rocprofv3's kernel-trace average)
        "roofline_vtrace": dict(roof("vtrace", vt_cold_ms) or {},
                                method=(f"HIP events around {VT_REPLAYS} back-to-back launches rotating over "
                                        f"{VT_COLD_SETS} disjoint input/output sets (cold: > 256 MB Infinity Cache)"),
                                warm={"launch_ms": round(vt_warm_ms, 5),
                                      "frac": round(work["vtrace"][1] / (vt_warm_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                      "method": f"{VT_REPLAYS} launches on the same resident tensors (cache-warm)"},
                                in_step_event_ms=round(kt["vtrace"]["ms"], 5) if "vtrace" in kt else None),
        # the whole step against its floors: stamped PMC bytes / the timed ms_per_step, and every
        # kernel's gap to max(HBM, MFMA) floor (freeimpala_amd/roofline.py)
        "step_roofline": dict(step_roofline(per_step, {k: v["count"] / max(1, args.profile_steps) for k, v in kt.items()},
                                            work, traffic, mfma, ms_per_step, dtype),
                              counters_file=counters_build.get("traffic_file")),
        # NOT a decomposition of ms_per_step: these come from the profiled pass after the timed loop
        "breakdown_source": {
            "fields": ["kernel_ms_per_step", "phase_ms", "step_roofline.kernels_by_gap"],
            "pass": (f"{args.profile_steps} profiled steps after the timed loop, a HIP event pair around "
                     "every launch (the events add a little time; the timed loop has none)"),
            "profiled_ms_per_step": round(sum(v for k, v in phases.items() if k != "steps"), 4),
            "timed_ms_per_step": round(ms_per_step, 4)},
        "kernel_ms_per_step": {k: round(v, 4) for k, v in sorted(per_step.items(), key=lambda x: -x[1])},
        "phase_ms": {k: round(v, 4) for k, v in phases.items() if k != "steps"},
        "final_loss": st["total_loss"], "grad_norm": st["grad_norm"],
        # RCCL's own view of the data-parallel communicator (ncclCommCount / ncclCommUserRank)
        "comm": L.comm_info(),
        "counters_build": counters_build,
    }
    if dp is not None:
        result["data_parallel"] = dp
    if rank == 0 and N == 1 and not args.no_cpu_baseline:
        # every core this process may use: the box's OMP_NUM_THREADS share when set (16 per GPU
        # on the pool's boxes, whose nproc counts the whole host), else the affinity mask
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or host_cpu_info()["affinity_cpus"] or 1
        try:
            full, why_not = full_cpu_step(args.arch, args.batch, args.cpu_full, args.cpu_sample,
                                          host_mem_headroom_gb())
            result["cpu_baseline"] = cpu_baseline(args.arch, T, A, args.cpu_seconds, threads, full=full)
            if why_not:
                result["cpu_baseline"]["full_step_skipped"] = why_not
            result["cpu_baseline"]["threads_basis"] = (
                "OMP_NUM_THREADS from the environment: the pool gives one GPU's job a 16-CPU share and "
                "sets OMP_NUM_THREADS=16 (nproc / the affinity mask count the whole host, shared with "
                "the node's other GPUs)" if os.environ.get("OMP_NUM_THREADS") else
                "the process affinity mask (no OMP_NUM_THREADS set)")
            result["speedup_vs_cpu"] = round(value / result["cpu_baseline"]["value"], 1)
        except Exception as e:  # the baseline is reported, never blocks the GPU number
            result["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    L.close()
    if ws > 1:
        dist.destroy_process_group()


def load_counters(arch, tba):
    """(traffic, mfma, info) from the newest profiles/*pmc_{traffic,mfma}_<arch>*.json whose
    _build.source_hash matches this tree; empty dicts when none does."""
    import glob
    from freeimpala_amd.build_info import runtime_key, source_hash
    h, rt = source_hash(), runtime_key()
    info = {"source_hash": h, "runtime": rt, "traffic_file": None, "mfma_file": None}
    if tba != (100, 4096, 18):
        return {}, {}, dict(info, note="counter passes exist for T=100 B=4096 A=18 only")

    def newest(kind):
        for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*pmc_{kind}_{arch}*.json")), reverse=True):
            try:
                with open(f) as fh:
                    d = json.load(fh)
            except (OSError, ValueError):
                continue
            b = d.get("_build", {})
            if b.get("source_hash") == h and b.get("runtime") == rt:  # same kernels, same switches
                return os.path.relpath(f, ROOT), {k: v for k, v in d.items() if not k.startswith("_")}
        return None, {}

    info["traffic_file"], tr = newest("traffic")
    info["mfma_file"], mf = newest("mfma")
    if not info["traffic_file"] and not info["mfma_file"]:
        info["note"] = "no counter pass stamped with this source hash and runtime: traffic / mfma_util_pmc null"
    return {k: v["hbm_bytes_per_launch"] for k, v in tr.items()}, mf, info


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
