"""bench.py --gpus N: the launch decision and the timed loop.

The driver runs `python bench.py --gpus N` with no launcher. bench.py must then start N ranks
itself (a child torch.distributed.run, decided before anything touches the GPU), refuse a GPU
count it cannot honour, and time each rank's own work apart from the barrier-bracketed time the
max over ranks is taken of. All of it runs on CPU here.
"""
import os
import socket
import subprocess
import sys

import pytest

from freeimpala_amd.launch import LaunchError, bench_launch_plan, timed_steps

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _plan(gpus, env, visible=8, argv=None):
    calls = []

    def vis():
        calls.append(1)
        return visible

    cmd = bench_launch_plan(gpus, env, argv if argv is not None else ["--gpus", str(gpus)], "/r/bench.py",
                            "/usr/bin/python3", vis, 29555)
    return cmd, len(calls)


def test_single_gpu_runs_in_process_without_counting_devices():
    assert _plan(1, {}) == (None, 0)


def test_gpus_n_without_launcher_spawns_n_ranks():
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    cmd, counted = _plan(8, {}, visible=8, argv=argv)
    assert counted == 1
    assert cmd[:3] == ["/usr/bin/python3", "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    # the ranks run the same script with the same arguments (so each sees --gpus 8 = WORLD_SIZE)
    assert cmd[-len(argv) - 1:] == ["/r/bench.py"] + argv


def test_too_few_devices_fails_loudly():
    with pytest.raises(LaunchError, match="needs 8 visible GPU"):
        _plan(8, {}, visible=1)
    with pytest.raises(LaunchError, match="needs 2 visible GPU"):
        _plan(2, {}, visible=0)


def test_one_device_rehearsal_needs_one_device():
    cmd, _ = _plan(2, {"FI_BENCH_DEVICE": "0", "FI_BENCH_NO_COMM": "1"}, visible=1)
    assert "--nproc-per-node=2" in cmd


def test_under_a_launcher_gpus_must_equal_world_size():
    assert _plan(2, {"WORLD_SIZE": "2", "LOCAL_RANK": "1"}) == (None, 0)
    with pytest.raises(LaunchError, match="disagrees"):
        _plan(8, {"WORLD_SIZE": "2", "LOCAL_RANK": "0"})
    with pytest.raises(LaunchError, match="disagrees"):  # torchrun --nproc-per-node 1 ... --gpus 2
        _plan(2, {"WORLD_SIZE": "1", "LOCAL_RANK": "0"})
    with pytest.raises(LaunchError):
        _plan(0, {})


def test_bench_gpus_n_on_a_box_without_n_devices_exits_nonzero():
    """The driver's command form: no 1-GPU line may come out of `--gpus N` on fewer devices
    (N = 64: more than any node has; here, with no GPU, --gpus 8 fails the same way)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "LOCAL_RANK", "RANK",
                                                               "TORCHELASTIC_RUN_ID", "FI_BENCH_DEVICE")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "64", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 2, r.stderr
    assert "needs 64 visible GPU" in r.stderr
    assert r.stdout.strip() == ""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _timed_worker(rank, world, port, out_dir):
    """bench.py's timed loop over gloo with rank 1 slower: the own times differ, the bracketed
    times (the max over ranks is taken of them) both cover the slow rank."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import json
    import time
    import torch.distributed as dist
    from freeimpala_amd import launch
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        delay = 0.01 if rank == 0 else 0.15
        own, br = launch.timed_steps(lambda: time.sleep(delay), lambda: None, dist.barrier, 4)
        per = launch.gather_objects({"ms_per_step": 1000 * own / 4, "allreduce_ms": 0.0})
        dp = launch.data_parallel_fields(per, grad_bytes=16, buckets=None)
        with open(os.path.join(out_dir, f"t{rank}.json"), "w") as fh:
            json.dump({"own": own, "bracketed": br, "dp": dp}, fh)
    finally:
        dist.destroy_process_group()


def test_rank_own_time_excludes_the_wait_for_the_slowest_rank(tmp_path):
    import json
    import torch.multiprocessing as mp
    mp.start_processes(_timed_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    t = [json.load(open(tmp_path / f"t{r}.json")) for r in range(2)]
    # 4 x 10 ms vs 4 x 150 ms (margins wide enough for a loaded CI host)
    assert t[0]["own"] < 0.3 and t[1]["own"] >= 0.6
    assert t[0]["bracketed"] >= 0.6                     # rank 0's bracket waits for rank 1
    per = t[0]["dp"]["rank_ms_per_step"]["per_rank"]
    assert per[1] > 2 * per[0]


def test_timed_steps_order():
    log = []
    own, br = timed_steps(lambda: log.append("s"), lambda: log.append("sync"), lambda: log.append("b"), 3)
    assert log == ["b", "s", "s", "s", "sync", "b"] and 0 <= own <= br


@pytest.mark.gpu
def test_bench_gpus2_spawns_two_ranks_on_the_gpu_box():
    """The driver's command form at N = 2 on a one-GPU box: `python bench.py --gpus 2` starts
    two ranks itself; FI_BENCH_DEVICE=0 pins both to the one device and FI_BENCH_NO_COMM skips
    the RCCL communicator (RCCL refuses two ranks on one device). One JSON line, n_gpus 2, the
    per-rank data_parallel fields."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "LOCAL_RANK", "RANK",
                                                               "TORCHELASTIC_RUN_ID")}
    env.update(FI_BENCH_DEVICE="0", FI_BENCH_NO_COMM="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--arch", "mlp",
                        "--steps", "3", "--warmup", "1", "--profile-steps", "1", "--sustain-seconds", "0.5",
                        "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * d["config"]["B_per_gpu"]
    dp = d["data_parallel"]
    assert dp["ranks"] == 2 and len(dp["rank_ms_per_step"]["per_rank"]) == 2
    assert "step_roofline" in d and d["breakdown_source"]["timed_ms_per_step"] == d["ms_per_step"]
    assert d["sustained"]["steps"] >= 1 and d["sustained"]["ms_per_step"] > 0
