"""GPU: the multi-GPU building blocks through the C ABI.

* a plan rebuilt from an exported row stage (bsmr_plan_export_rows / bsmr_plan_import_rows, the
  row stage rank 0 broadcasts) has every RPHM/BSMR array and statistic of the original plan;
* bsmr_sddmm_panels_local (a shard with only its own A rows) writes exactly its panels' outputs,
  and the shards together give the oracle's values (checkData rule);
* bench.py's sharded path run as 2 fresh processes on the one GPU (gloo: RCCL refuses two ranks
  on one device): global plan, row-stage broadcast, local A, B broadcast, P gather, checkData.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as O
from bsmr import Plan, RowStage, make_data, synth
from bsmr import dist as D
from gpu_util import PLAN_ARRAYS, half_values, torch_cuda

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FREE = 288 * 1024 ** 3


def _cases():
    return {
        "zipf": synth.random_rows(517, 4000, 60, seed=2, zipf=1.1, empty_frac=0.05),
        "blocky": synth.block_mask(512, 16, 0.15, seed=4),
        "banded": synth.banded_fem_like(6000, 22, seed=5, band=48),
    }


@pytest.mark.parametrize("name", ["zipf", "blocky", "banded"])
@pytest.mark.parametrize("via", ["host", "device"])
def test_import_rows_reproduces_plan(name, via):
    torch = torch_cuda()
    M, N, rp, ci = _cases()[name]
    a = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    hdr, rows = a.export_rows()
    assert hdr.num_reordered_rows == len(rows) == a.stats()["num_reordered_rows"]
    # the header survives its byte form (what the broadcast ships)
    hdr2 = RowStage.from_array(hdr.to_array())
    assert hdr2.as_dict() == hdr.as_dict()
    if via == "device":
        d = torch.from_numpy(rows.view(np.int32)).cuda()
        b = Plan.from_row_stage(rp, ci, hdr2, d.data_ptr(), delta=0.3)
    else:
        b = Plan.from_row_stage(rp, ci, hdr2, rows, delta=0.3)
    for arr in PLAN_ARRAYS:
        assert np.array_equal(a.array(arr), b.array(arr)), arr
    sa, sb = a.stats(), b.stats()
    for k in ("num_clusters", "num_row_panels", "num_dense_tiles", "num_residual",
              "max_dense_tiles_per_panel", "num_sparse_thread_blocks", "block_size"):
        assert sa[k] == sb[k], k
    assert a.evaluate() == b.evaluate()
    # the imported plan recolumns like the original
    a.recolumn(0.0)
    b.recolumn(0.0)
    for arr in PLAN_ARRAYS:
        assert np.array_equal(a.array(arr), b.array(arr)), arr


def test_import_rows_rejects_bad_rows():
    M, N, rp, ci = _cases()["zipf"]
    a = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    hdr, rows = a.export_rows()
    bad = rows.copy()
    bad[1] = bad[0]  # a row twice
    with pytest.raises(Exception):
        Plan.from_row_stage(rp, ci, hdr, bad)
    bad = rows.copy()
    bad[0] = M  # out of range
    with pytest.raises(Exception):
        Plan.from_row_stage(rp, ci, hdr, bad)
    # an inflated zero-row count with one non-empty row dropped: R + z == M still holds and the
    # rows are distinct and non-empty, but a row of S would never be computed
    h2 = RowStage.from_array(hdr.to_array())
    h2.num_zero_rows += 1
    h2.num_reordered_rows -= 1
    with pytest.raises(Exception, match="num_zero_rows"):
        Plan.from_row_stage(rp, ci, h2, rows[1:].copy())
    # column-stage geometry not derived from N
    for field, v in (("block_size", 0), ("num_blocks_per_row", hdr.num_blocks_per_row + 1),
                     ("cluster_block_dim", hdr.cluster_block_dim + 32)):
        h3 = RowStage.from_array(hdr.to_array())
        setattr(h3, field, v)
        with pytest.raises(Exception, match="inconsistent"):
            Plan.from_row_stage(rp, ci, h3, rows)


def _run_local(plan, rows, A, B, K, nnz, shards, dtype):
    torch = torch_cuda()
    tdt = {0: torch.float32, 1: torch.float16, 2: torch.bfloat16}[dtype]
    dB = torch.from_numpy(B).cuda().to(tdt)
    dP = torch.full((nnz,), float("nan"), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    keep = []
    for p0, p1 in shards:
        if p0 == p1:
            continue
        Al = D.shard_a_rows(A, K, rows, p0, p1)
        dA = torch.from_numpy(Al.reshape(-1)).cuda().to(tdt)
        keep.append(dA)
        plan.sddmm_panels_local(dA.data_ptr(), dB.data_ptr(), K, dP.data_ptr(), p0, p1,
                                stream=s, dtype=dtype)
    torch.cuda.synchronize()
    return dP.cpu().numpy()


@pytest.mark.parametrize("name,K,dtype,world", [
    ("zipf", 128, 0, 3), ("zipf", 64, 0, 2), ("zipf", 32, 0, 4), ("zipf", 256, 1, 3),
    ("zipf", 512, 2, 2), ("blocky", 256, 1, 2), ("banded", 128, 0, 1), ("banded", 256, 1, 2),
    ("zipf", 512, 0, 5),
])
@pytest.mark.parametrize("staged", ["0", "1"])
def test_panels_local_every_output_once(name, K, dtype, world, staged):
    """Each shard writes exactly its panels' entries from its own A rows (NaN elsewhere stays
    NaN); together they equal the oracle. world 1 on the banded case: the whole range, whose
    plan-wide layout uses original-order row blocks, runs the reordered layout instead. staged:
    results through LDS in CSR order (BSMR_OUT_STAGED) or one store per entry."""
    M, N, rp, ci = _cases()[name]
    # (the blocky mask is tile-dominated: its auto launch is column-major, so force row blocks)
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE,
                layout="rowblock" if name == "blocky" else "auto",
                tuning={"out_staged": int(staged)})
    rows = plan.array("reorderedRows")
    shards = [plan.shard(K, r, world, dtype) for r in range(world)]
    A = make_data(M * K)
    B = make_data(N * K)
    Ar, Br = (A, B) if dtype == 0 else (half_values(A, dtype), half_values(B, dtype))
    ref = O.sddmm_cpu(O.CSR.from_arrays(M, N, rp, ci), K, Ar, Br)
    P = _run_local(plan, rows, A, B, K, len(ci), shards, dtype)
    assert np.isfinite(P).all()
    assert O.check_data(ref, P) == 0
    for p0, p1 in shards:
        part = _run_local(plan, rows, A, B, K, len(ci), [(p0, p1)], dtype)
        mine = np.zeros(len(ci), bool)
        for r in rows[16 * p0:16 * p1]:
            mine[rp[r]:rp[r + 1]] = True
        assert np.isfinite(part[mine]).all() and np.isnan(part[~mine]).all(), (p0, p1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(600)
@pytest.mark.parametrize("extra", [["--config", "C2", "--strong", "off"],
                                   ["--config", "C2", "--shard", "global", "--strong", "off"],
                                   ["--config", "C2", "--strong-scale", "0.05"],
                                   ["--config", "C4", "--scale", "0.05"],
                                   ["--config", "C4", "--scale", "0.05", "--shard", "global"]])
def test_bench_sharded_two_ranks_one_gpu(extra):
    """bench.py's multi-GPU path in 2 fresh processes sharing the GPU (a rehearsal of the
    driver's torchrun launch; times are not a measurement): the gathered P passes checkData."""
    env = dict(os.environ, BSMR_DIST_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=540, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    out = json.loads(line[0])
    assert out["n_gpus"] == 2 and out["checkData_errors_gathered_P"] == 0
    sh = out["shards"]
    assert sum(sh["entries"]) == out["config"]["nnz"]
    if out["config"].get("shard_mode") == "local":  # contiguous original row panels
        assert sum(sh["rows"]) == out["config"]["M"] and min(sh["rows"]) > 0
        if "C2" in extra:  # exactly the two stacked copies
            assert sh["rows"] == [out["config"]["M"] // 2] * 2
            assert sh["entries"][0] == sh["entries"][1]
    else:
        assert sum(sh["panels"]) == out["config"]["num_row_panels"]
        assert min(sh["panels"]) > 0
    assert out["scaling"] == ("weak" if "C2" in extra else "strong")
    # the weak-scaling value says what it is: independent per-rank replicas of C2
    assert ("independent replicas" in out.get("scaling_detail", "")) == ("C2" in extra)
    if "--strong-scale" in extra:  # the default N > 1 line carries the north_star reddit split
        sc = out["strong_C4"]
        for split in ("global", "local"):
            assert "error" not in sc[split], sc[split]
            assert sc[split]["checkData_errors_gathered_P"] == 0, split
            assert len(sc[split]["shards"]["ms_per_step"]) == 2
    else:
        assert "strong_C4" not in out


@pytest.mark.timeout(600)
def test_bench_sharded_rccl_one_rank():
    """bench.py's multi-GPU path on RCCL (backend "nccl"), launched by torchrun before any GPU
    call, at world size 1 (--force-sharded: RCCL refuses two ranks on one device): RCCL init, the
    device-tensor broadcasts (B, row stage, the strong_C4 pattern), the compact P gather and the
    segment gather all execute on MI355X; both strong_C4 splits and the C2 line pass checkData."""
    env = dict(os.environ, OMP_NUM_THREADS="8")
    env.pop("BSMR_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--force-sharded", "--steps", "5",
           "--warmup", "2", "--strong", "on", "--strong-scale", "0.1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=540, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    out = json.loads(line[0])
    assert out["config"]["backend"] == "nccl"
    assert out["n_gpus"] == 1 and out["checkData_errors_gathered_P"] == 0
    sc = out["strong_C4"]
    for split in ("global", "local"):
        assert "error" not in sc[split], sc[split]
        assert sc[split]["checkData_errors_gathered_P"] == 0, split
        assert sc[split]["ms_per_step"] > 0
    assert sc["global"]["whole_plan_one_gpu"]["ms_per_step"] > 0
    assert sum(sc["global"]["shards"]["entries"]) == sc["nnz"]


@pytest.mark.timeout(600)
def test_bench_self_launch_force_sharded_one_gpu():
    """`bench.py --gpus 1 --force-sharded` with no launcher: bench starts torch.distributed.run as
    a child (the same path `--gpus 8` takes on the driver's node) and the line reports the ranks
    that ran, with the strong_C4 block of the north_star split."""
    env = dict(os.environ, OMP_NUM_THREADS="8")
    for k in ("BSMR_DIST_BACKEND", "WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--force-sharded",
           "--steps", "5", "--warmup", "2", "--strong", "on", "--strong-scale", "0.05",
           "--no-vendor", "--pmc", "off"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=540, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "torch.distributed.run" in r.stderr
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, r.stdout[-2000:]
    out = json.loads(line[0])
    assert out["n_gpus"] == 1 and out["config"]["backend"] == "nccl"
    assert out["checkData_errors_gathered_P"] == 0
    for split in ("global", "local"):
        assert out["strong_C4"][split]["checkData_errors_gathered_P"] == 0, split


def test_shard_rebalance_moves_cuts_toward_measured_balance():
    """bsmr_plan_shard_rebalance: cuts stay on row-block boundaries, span [0, P], do not move
    when every shard took the same time per model cost, and shrink a shard that ran slow."""
    M, N, rp, ci = synth.random_rows(4000, 6000, 60, seed=31, zipf=1.1)
    K = 128
    plan = Plan(M, N, rp, ci, alpha=0.3, delta=0.3, free_mem_bytes=FREE)
    world = 4
    P = plan.stats()["num_row_panels"]
    cuts = [plan.shard(K, r, world)[0] for r in range(world)] + [P]
    assert cuts[0] == 0 and all(a <= b for a, b in zip(cuts, cuts[1:]))
    rb = plan.stats()["rb_rows"][2] // 16  # panels per row block (512-byte rows)
    assert rb > 0 and all(c % rb == 0 or c == P for c in cuts)
    same = plan.shard_rebalance(K, world, cuts, [1.0] * world)
    # equal times on model-balanced shards: the cuts can only move by the rounding to row blocks
    assert all(abs(a - b) <= rb for a, b in zip(same, cuts)) and same[0] == 0 and same[-1] == P
    slow = plan.shard_rebalance(K, world, cuts, [2.0, 1.0, 1.0, 1.0])
    assert slow[1] <= cuts[1] and slow[-1] == P
    assert all(c % rb == 0 or c == P for c in slow)
    assert all(a <= b for a, b in zip(slow, slow[1:]))
    # unmeasured shards (time 0 / NaN) keep their model cost: with the measured ones at equal
    # time per model cost (real ms-scale values, far from 1.0), the cuts stay at the model cut
    for ms in ([0.0012, 0.0, 0.0012, float("nan")], [0.0, 0.0012, float("inf"), 0.0012]):
        kept = plan.shard_rebalance(K, world, cuts, ms)
        assert all(abs(a - b) <= rb for a, b in zip(kept, cuts)), (ms, kept, cuts)
    with pytest.raises(Exception):
        plan.shard_rebalance(K, world, cuts[:-1] + [P - 1], [1.0] * world)
