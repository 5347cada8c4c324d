"""The multi-GPU path on CPU: two ranks over gloo run exactly the code bench.py runs over RCCL
(batchreactor.jl_amd/shard.py: contiguous per-rank slices of the ensemble, no collective during
the integration, one all-gather of final states + counters, max-over-ranks time). The per-rank
compute is the CPU oracle here (no GPU); the gathered ensemble must equal a single-process run
over the whole range, in order.
"""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PER_RANK = 3
TF = 2e-3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _inputs(pkg, start, count):
    from batchreactor_amd import ensemble
    m = pkg.Mechanism.from_files(os.path.join(ROOT, "tests", "golden", "lib"), gas_mech="h2o2.dat")
    return m, ensemble.make_inputs(m, "h2o2", start, count)


def _oracle_run(m, T, Asv, U0):
    import oracle
    lib = os.path.join(ROOT, "tests", "golden", "lib")
    om = oracle.Mech(os.path.join(lib, "h2o2.dat"), os.path.join(lib, "therm.dat"))
    U, st, _ = om.integrate_batch(T, Asv, U0, np.full(len(T), TF), analytic_jac=True, nthreads=1)
    S = np.array([[s["nsteps"], s["nfe"], s["status"]] for s in st], dtype=np.float64)
    return U, S


def _rank_strong(rank, world, port, out_dir, total):
    """strong scaling: `total` reactors split over the ranks (slices differ in length by one)"""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist
    import _pkgload
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = _pkgload.load()
    from batchreactor_amd import shard
    start, stop = shard.shard_range(rank, world, total)
    m, (T, Asv, U0) = _inputs(pkg, start, stop - start)
    U, S = _oracle_run(m, T, Asv, U0)
    Ug, Sg = shard.gather_ensemble(torch.from_numpy(U), torch.from_numpy(S), dist, total)
    np.save(os.path.join(out_dir, f"SU{rank}.npy"), Ug.numpy())
    np.save(os.path.join(out_dir, f"SS{rank}.npy"), Sg.numpy())
    dist.destroy_process_group()


def _rank(rank, world, port, out_dir):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch
    import torch.distributed as dist
    import _pkgload
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pkg = _pkgload.load()
    from batchreactor_amd import shard
    start, stop = shard.shard_slice(rank, PER_RANK)
    m, (T, Asv, U0) = _inputs(pkg, start, stop - start)
    U, S = _oracle_run(m, T, Asv, U0)
    t = shard.max_over_ranks(0.5 + rank, dist)
    Ug, Sg = shard.gather_ensemble(torch.from_numpy(U), torch.from_numpy(S), dist)
    np.save(os.path.join(out_dir, f"U{rank}.npy"), Ug.numpy())
    np.save(os.path.join(out_dir, f"S{rank}.npy"), Sg.numpy())
    np.save(os.path.join(out_dir, f"t{rank}.npy"), np.array([t]))
    dist.destroy_process_group()


def test_two_rank_gloo_shard_and_gather(pkg, orc, tmp_path):
    world = 2
    mp.start_processes(_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    m, (T, Asv, U0) = _inputs(pkg, 0, world * PER_RANK)
    U, S = _oracle_run(m, T, Asv, U0)
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"U{r}.npy"), U)   # same inputs, same order
        np.testing.assert_array_equal(np.load(tmp_path / f"S{r}.npy"), S)
        assert float(np.load(tmp_path / f"t{r}.npy")[0]) == 0.5 + (world - 1)


def test_strong_scaling_slices_cover_the_ensemble(pkg):
    """shard_range: contiguous slices in ensemble order, sizes within one, union = [0, total),
    for the BASELINE 1e5 ensemble over 1/2/4/8 GPUs and ragged totals."""
    from batchreactor_amd import shard
    for total in (100000, 7, 12345, 3):
        for world in (1, 2, 3, 4, 8):
            r = [shard.shard_range(k, world, total) for k in range(world)]
            assert r[0][0] == 0 and r[-1][1] == total
            assert all(r[k][1] == r[k + 1][0] for k in range(world - 1))
            sizes = [b - a for a, b in r]
            assert max(sizes) - min(sizes) <= 1


def test_two_rank_gloo_strong_scaling(pkg, orc, tmp_path):
    """Strong scaling over two gloo ranks with an odd total (slices of 3 and 2 reactors): the
    gathered ensemble equals a single-process run over the whole range, in order."""
    world, total = 2, 5
    mp.start_processes(_rank_strong, args=(world, _free_port(), str(tmp_path), total), nprocs=world, join=True,
                       start_method="spawn")
    m, (T, Asv, U0) = _inputs(pkg, 0, total)
    U, S = _oracle_run(m, T, Asv, U0)
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"SU{r}.npy"), U)
        np.testing.assert_array_equal(np.load(tmp_path / f"SS{r}.npy"), S)


def _bench(*args, env_extra=None):
    import json
    import subprocess
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


def test_bench_spawns_ranks_for_gpus_n():
    """bench.py --gpus 2 without a launcher spawns two rank processes itself (before any GPU call);
    the dry-run path runs the same launch and sharding over gloo on the CPU: n_gpus is the world
    size the process group reports, and the two contiguous slices split the 1e5 GRI ensemble."""
    rc, line, err = _bench("--gpus", "2", "--dry-run")
    assert rc == 0, err
    assert line["n_gpus"] == 2 and line["total_reactors"] == 100000
    assert line["slices"] == [[0, 50000], [50000, 100000]]
    rc, line, err = _bench("--gpus", "2", "--dry-run", "--scaling", "weak", "--n", "1000")
    assert rc == 0 and line["slices"] == [[0, 1000], [1000, 2000]]


def test_bench_rejects_world_size_mismatch():
    """--gpus N that disagrees with the launcher's world size exits non-zero (no line printed)."""
    rc, line, _ = _bench("--gpus", "2", "--dry-run", env_extra={"WORLD_SIZE": "1"})
    assert rc != 0 and line is None
