"""CPU tests of bench.py's launch contract (no GPU; BSMR_BENCH_PROBE=1 makes each rank report its
rank / world and stop before any device call):

* `bench.py --gpus 2` with no launcher starts torch.distributed.run with 2 ranks as a child process
  (never an exec from a process that touched HIP) and exits with its return code, so a driver's
  `--gpus N` always times N ranks;
* a launcher whose WORLD_SIZE differs from --gpus is refused (non-zero exit), so the line's n_gpus
  can never disagree with the ranks that ran;
* `--gpus 1` stays in-process.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = dict(os.environ, BSMR_BENCH_PROBE="1", BSMR_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(kw)
    return env


def _probes(stdout):
    return [json.loads(x) for x in stdout.splitlines() if x.startswith("{")]


def test_gpus_2_self_launches_two_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "3", "--warmup", "1"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    p = _probes(r.stdout)
    assert sorted(x["rank"] for x in p) == [0, 1], r.stdout
    assert all(x["world"] == 2 and x["gpus"] == 2 and x["self_launched"] for x in p)
    assert "torch.distributed.run" in r.stderr


def test_gpus_1_stays_in_process():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"], capture_output=True, text=True,
                       timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    p = _probes(r.stdout)
    assert len(p) == 1 and p[0]["world"] == 1 and not p[0]["self_launched"]


def test_world_size_mismatch_fails():
    env = _env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"], capture_output=True, text=True,
                       timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and not _probes(r.stdout)


def test_child_failure_propagates():
    """A rank that fails makes the self-launch fail: the parent exits with the launcher's code."""
    env = _env(WORLD_SIZE="", BSMR_BENCH_PROBE="0")
    env.pop("WORLD_SIZE")
    # --K 7 is rejected by the library on every rank (K must be a multiple of 16); gloo ranks on
    # a CPU-only host fail even earlier (no device): either way a non-zero exit
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--K", "7", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline", "--no-vendor", "--pmc", "off"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode != 0


def test_cpu_leg_pins_one_thread_per_core_in_the_affinity_set():
    """BASELINE.md §2's OMP_PROC_BIND=close for the CPU leg: bench.close_cpus lists CPUs of the
    start-up affinity set, distinct, physical cores (one SMT sibling each) first, in order."""
    sys.path.insert(0, ROOT)
    import bench

    aff = set(bench.AFFINITY)
    for n in (1, 2, len(aff), len(aff) + 3):
        cpus = bench.close_cpus(n)
        assert len(cpus) == min(max(n, 1), len(aff))
        assert len(set(cpus)) == len(cpus) and set(cpus) <= aff
    assert 1 <= bench.host_threads() <= len(aff)
