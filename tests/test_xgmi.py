"""The one-shot xGMI exchange (psg_xgmi_*) and the node barrier.

The barrier test runs on CPU.  The exchange test runs 2 and 3 rank PROCESSES
on one MI355X: each maps the others' request vectors and shards through hipIpc
handles (on one GPU the "peer" reads stay on the card; on the 8-GPU node they
cross xGMI), so the protocol — handle exchange, offsets, rank-order sums,
barriers — is exercised end to end and checked against the oracle.
"""
import multiprocessing as mp
import os
import sys
import uuid

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _paths():
    for p in (os.path.join(ROOT, "parameter-server_amd", "python"), os.path.join(ROOT, "oracle")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _barrier_rank(name, world, rank, rounds, out):
    _paths()
    import psg
    b = psg.NodeBarrier(name, world, rank)
    for _ in range(rounds):
        b.wait(30.0)
    b.close()
    out.put(rank)


def test_node_barrier_cpu():
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    name = "psg_test_" + uuid.uuid4().hex[:12]
    procs = [ctx.Process(target=_barrier_rank, args=(name, 3, r, 200, out)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(60)
    assert all(p.exitcode == 0 for p in procs)
    assert sorted(out.get(timeout=5) for _ in range(3)) == [0, 1, 2]


def _xgmi_rank(rank, world, n, steps, name, q_in, q_out, mode=0, write=False):
    _paths()
    import oracle
    import psg
    # one GPU per rank where the box has them (the reads then cross xGMI); on a
    # 1-GPU box the ranks share it and the peer reads stay on the card
    psg.set_device(rank % psg.device_count())
    blk = n // world
    vals = psg.DeviceBuffer(n * 4)
    lo_v, hi_v = (0.0, 1000.0) if mode == 0 else (-1.0, 1.0)
    vals.fill_synth(n, psg.F32, 7 + rank, mode, lo_v, hi_v)
    store = psg.Store(psg.DENSE, psg.F32, rank * blk, (rank + 1) * blk, blk)
    sptr = store.info().vals
    out = psg.DeviceBuffer(n * 4)
    psg.device_sync()
    q_out.put(("h", rank, psg.ipc_export(vals.ptr), psg.ipc_export(sptr), psg.ipc_export(out.ptr)))
    handles = q_in.get(timeout=120)
    vptrs = [vals.ptr if r == rank else psg.ipc_open(handles[r][0]) for r in range(world)]
    sptrs = [sptr if r == rank else psg.ipc_open(handles[r][1]) for r in range(world)]
    optrs = [out.ptr if r == rank else psg.ipc_open(handles[r][2]) for r in range(world)]
    x = psg.Xgmi(world, rank, vptrs, sptrs)
    x.set_outs(optrs)
    bar = psg.NodeBarrier(name, world, rank)
    bar.wait()
    for _ in range(steps):
        x.push(store, n)
        if write:
            # no barrier between the phases: this rank's own Push is done
            x.pull_write(store, n)
            psg.device_sync()
            bar.wait()
            continue
        psg.device_sync()
        bar.wait()
        x.pull(store, out, n)
        psg.device_sync()
        bar.wait()
    got = out.download(np.float32, n)
    exp = np.zeros(n, np.float32)
    ref = [oracle.synth(n, oracle.F32, 7 + w, mode, lo_v, hi_v) for w in range(world)]
    for r in range(world):  # shard r: `steps` pushes of every worker, in rank order
        st = oracle.Store(oracle.F32)
        lo = r * blk
        for _ in range(steps):
            for w in range(world):
                st.handle(oracle.PUSH, None, ref[w][lo:lo + blk], blk, first_key=lo)
        exp[lo:lo + blk] = st.handle(oracle.PULL, None, None, blk, first_key=lo)
    ok = bool(np.array_equal(got, exp))
    bar.wait()  # nobody unmaps a buffer a peer still reads
    x.close()
    for r in range(world):
        if r != rank:
            psg.ipc_close(vptrs[r])
            psg.ipc_close(sptrs[r])
            psg.ipc_close(optrs[r])
    bar.close()
    q_out.put(("r", rank, ok))


@pytest.mark.gpu
@pytest.mark.parametrize("world,mode,write", [(2, 0, False), (3, 0, False), (2, 1, False), (3, 1, False),
                                              (2, 0, True), (3, 1, True)])
def test_xgmi_exchange_multiprocess(world, mode, write):
    """Every rank's Push lands on every shard and every Pull reads every shard.
    mode 0: integer-valued data (the reference KATs); mode 1: real-valued
    U(-1, 1).  k_xgmi_push adds the sources to the shard one at a time in rank
    order, which is the oracle's order of sequential pushes, so both are
    bit-exact (no 1e-6 tolerance needed)."""
    n = 3 * 64 * 4096  # divisible by 2 and 3, 16-B blocks
    ctx = mp.get_context("spawn")
    q_out = ctx.Queue()
    q_in = [ctx.Queue() for _ in range(world)]
    name = "psg_xgmi_" + uuid.uuid4().hex[:12]
    procs = [ctx.Process(target=_xgmi_rank, args=(r, world, n, 3, name, q_in[r], q_out, mode, write))
             for r in range(world)]
    for p in procs:
        p.start()
    handles = {}
    for _ in range(world):
        tag, r, hv, hs, ho = q_out.get(timeout=240)
        handles[r] = (hv, hs, ho)
    for r in range(world):
        q_in[r].put(handles)
    results = [q_out.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert all(ok for _, _, ok in results), results


@pytest.mark.gpu
@pytest.mark.parametrize("nproc,exchange", [(2, None), (2, "xgmiw/0"), (3, "xgmiw/2")])
def test_bench_shared_gpu_xgmi_verified(nproc, exchange):
    """bench.py's N>1 path end to end with its ranks on one GPU
    (PSG_BENCH_SHARE_GPU=1: the xGMI exchange, no RCCL): the calibration's
    checksum verification of the pulled shards must pass and the closed-form
    parity check must hold after every push the run made.  Forced: the Pull as
    writes (xgmiw/0), and that form double-buffered on two streams over
    ragged chunks (xgmiw/2 at 3 ranks)."""
    import json
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PSG_BENCH_SHARE_GPU="1")
    if exchange:
        env["PSG_BENCH_EXCHANGE"] = exchange
    keys = 3 * (1 << 20) + 3 * 4 * 37 if nproc == 3 else 1 << 22
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--keys", str(keys),
           "--steps", "3", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == nproc and res["parity_check"] is True, res
    assert res["config"].get("xgmi_checksum_verified") is True, res
    if exchange:
        assert "as writes" in res["config"]["exchange"], res["config"]


def test_node_barrier_timeout_poisons_and_names_are_exclusive():
    """A wait that times out breaks the barrier for every rank (its arrival was
    already counted, so a later wait must not release a phase early), and
    rank 0 refuses a name whose segment already exists (a crashed job's)."""
    _paths()
    import psg
    name = "psg_test_" + uuid.uuid4().hex[:12]
    b0 = psg.NodeBarrier(name, 2, 0)
    b1 = psg.NodeBarrier(name, 2, 1)
    with pytest.raises(psg.PsgError, match="timed out"):
        b0.wait(0.05)  # rank 1 never arrives
    with pytest.raises(psg.PsgError, match="broken"):
        b1.wait(1.0)
    with pytest.raises(psg.PsgError, match="broken"):
        b0.wait(1.0)
    with pytest.raises(psg.PsgError, match="O_EXCL"):
        psg.NodeBarrier(name, 2, 0)  # the segment still exists
    b1.close()
    b0.close()
    b2 = psg.NodeBarrier(name, 1, 0)  # unlinked by rank 0's close: the name is free again
    b2.wait(1.0)
    b2.close()
