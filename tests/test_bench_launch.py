"""bench.py's multi-rank launch (VERDICT r3 "next" 1): `--gpus N` from a plain
shell must run N rank processes itself, or fail; never a silent 1-rank line.

CPU tests run the launcher with `--launch-check` (the rendezvous alone, no GPU
work), from a plain shell and under torchrun; the GPU
test runs the real sharded bench with 2 ranks sharing the box's one GPU
through the library's host all-reduce transport (RCCL refuses one GPU twice)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def _json_lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_spawns_n_ranks(n):
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--launch-check"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert p.returncode == 0, p.stderr[-2000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout  # rank 0 only
    assert lines[0]["n_gpus"] == n and lines[0]["ranks_counted"] == n


def test_torchrun_launch_runs_torch_free_workers():
    """The driver's N > 1 launch (`python -m torch.distributed.run ...
    bench.py --gpus N`): each torchrun rank joins gloo on the CPU only to
    publish rank 0's rendezvous port and runs its work in a child that never
    imports torch (tritd.rendezvous)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), BENCH, "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=240, env=_env())
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_counted"] == 2
    assert lines[0]["torch_in_workers"] is False


def test_world_size_mismatch_fails_loudly():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=120, env=_env(WORLD_SIZE="1"))
    assert p.returncode != 0
    assert "does not match WORLD_SIZE" in p.stderr


def test_single_gpu_needs_no_launcher():
    p = subprocess.run([sys.executable, BENCH, "--launch-check"], capture_output=True, text=True,
                       timeout=120, env=_env())
    assert p.returncode == 0, p.stderr[-2000:]
    assert _json_lines(p.stdout)[0]["n_gpus"] == 1


@pytest.mark.gpu
def test_bench_two_ranks_from_plain_shell():
    """The whole sharded bench, 2 ranks, started as `python3 bench.py --gpus 2`."""
    p = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "2", "--comm", "host", "--no-cpu",
                        "--no-e2e", "--n", "64", "--steps", "4", "--warmup", "1"],
                       capture_output=True, text=True, timeout=600, env=_env())
    assert p.returncode == 0, p.stderr[-4000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    line = lines[0]
    assert line["n_gpus"] == 2
    assert line["comm"] == {"transport": "host", "nranks": 2}
    assert line["hip_runtimes_mapped"] == 1 and "/opt/rocm" in line["hip_runtime"]
    assert line["value"] > 0 and line["rre_final"] < 1e-3
    # the per-rank breakdown: each rank's rows, iteration,
    # all-reduce and compute ms, two all-reduces per iteration
    pr = line["per_rank"]
    assert [p["rank"] for p in pr] == [0, 1] and sum(p["rows"] for p in pr) == 64
    for p in pr:
        assert p["allreduces_per_iteration"] == 2
        assert 0 < p["allreduce_ms"] < p["iteration_ms"]
        assert abs(p["compute_ms"] + p["allreduce_ms"] - p["iteration_ms"]) < 1e-9


@pytest.mark.gpu
def test_bench_two_ranks_under_torchrun():
    """The driver's own N > 1 command shape (`python -m torch.distributed.run
    --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P
    bench.py --gpus N ...`), 2 ranks sharing the box's GPU over the host
    transport: torchrun's rank processes publish the rendezvous port over gloo
    and run the GPU work in torch-free workers; the line reports one HIP / HSA
    / RCCL copy each, from /opt/rocm, in rank 0's worker."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), BENCH, "--gpus", "2", "--comm", "host", "--no-cpu", "--no-e2e",
                        "--side", "64", "--steps", "4", "--warmup", "1"],
                       capture_output=True, text=True, timeout=600, env=_env())
    assert p.returncode == 0, p.stderr[-4000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["comm"] == {"transport": "host", "nranks": 2}
    assert line["value"] > 0 and line["rre_final"] < 1e-3
    st = line["runtime_stack"]
    assert all(len(v) == 1 and v[0].startswith("/opt/rocm") for v in st.values()), st
