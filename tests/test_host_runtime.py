"""The C++ host runtime (ps:: API, local Van, slicer, merge, barriers) on CPU.

tests/_bin/kv_cluster_host runs real KVWorker / KVServer nodes with a host
request handle (test code), so no GPU is needed.  The reference's own harnesses
compiled unmodified against the runtime live in tests/_dropin/ (built by
`make -C parameter-server_amd dropin` where the reference tree exists).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "_bin")
DROPIN = os.path.join(ROOT, "tests", "_dropin")


def run(path, *args, timeout=120, env=None):
    e = dict(os.environ)
    if "-procs" in map(str, args):
        # a process job still running 15 s before the test's limit is hung: the
        # launcher has every node print the stacks of all its threads (SIGQUIT)
        # and kills the job, so the failure says where it stopped
        e["PS_JOB_TIMEOUT_S"] = str(max(5, timeout - 15))
    if env:
        e.update(env)
    r = subprocess.run([path, *map(str, args)], capture_output=True, text=True, timeout=timeout, env=e)
    if r.returncode == 124 and "PS_JOB_TIMEOUT_S" in r.stderr:
        # the whole dump, not a tail: which node waits where is the evidence
        print(r.stderr)
    return r


def _need(path):
    if not os.path.exists(path):
        pytest.skip(f"{path} not built (make -C parameter-server_amd all)")


def test_svector_semantics():
    """SVector copy/share/Slice/detach/reinterpret semantics (SVector_test.cpp)."""
    exe = os.path.join(BIN, "svector_unit")
    _need(exe)
    r = run(exe)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "svector ok" in r.stdout


def test_receive_queue_conditional_pop():
    """The receive queue's PopIf (internal/customer.h), which the servers'
    gather window relies on: an empty queue is no refusal, a rejected head is,
    a message pushed while a consumer polls is taken (never reported as a
    refusal), and messages leave in priority then arrival order."""
    exe = os.path.join(BIN, "queue_unit")
    _need(exe)
    r = run(exe)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "queue ok" in r.stdout


def test_shm_frame_arena():
    """The process-mode frame arena (src/shm_pool.cc): live frames never
    overlap under random churn, freed ranges coalesce, a full arena and an
    oversized frame fall back to blocks of their own, a peer's mapping by name
    shows a frame's bytes, and nothing is left in /dev/shm."""
    exe = os.path.join(BIN, "shm_arena_unit")
    _need(exe)
    before = {f for f in os.listdir("/dev/shm") if f.startswith("psg.")}
    r = run(exe, env={"PS_SHM_ARENA_MB": "16"})
    assert r.returncode == 0, r.stderr[-2000:]
    assert "shm arena ok" in r.stdout
    after = {f for f in os.listdir("/dev/shm") if f.startswith("psg.")}
    assert after <= before, sorted(after - before)


@pytest.mark.parametrize("ns,nw", [(1, 1), (2, 1), (3, 2), (8, 4)])
def test_host_cluster(ns, nw):
    exe = os.path.join(BIN, "kv_cluster_host")
    _need(exe)
    r = run(exe, "-ns", ns, "-nw", nw)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count(" ok") == nw


def test_num_nodes_from_environment():
    exe = os.path.join(BIN, "kv_cluster_host")
    _need(exe)
    r = run(exe, env={"PS_NUM_SERVER": "2", "PS_NUM_WORKER": "3"})
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count(" ok") == 3


def test_dropin_connection():
    """tests/test_connection.cpp of the reference, unmodified: Start / Finalize only."""
    exe = os.path.join(DROPIN, "test_connection")
    _need(exe)
    for ns, nw in [(1, 1), (2, 3)]:
        r = run(exe, "-ns", ns, "-nw", nw)
        assert r.returncode == 0, r.stderr[-2000:]


def _has_gpu():
    try:
        import psg
        return psg.device_count() > 0
    except Exception:
        return False


def test_default_handle_fails_loudly_without_gpu():
    """The HBM store has no CPU fallback: with no GPU the server's CHECK aborts the job."""
    exe = os.path.join(DROPIN, "test_kv_app")
    _need(exe)
    if _has_gpu():
        pytest.skip("a GPU is present")
    r = run(exe, "-ns", 1, "-nw", 1, timeout=60)
    assert r.returncode != 0
    assert "value store lives in HBM" in r.stderr


# ---- process mode: one node per OS process (src/tcp_van.cc) ------------------
@pytest.mark.parametrize("ns,nw", [(1, 1), (2, 3)])
def test_dropin_connection_processes(ns, nw):
    exe = os.path.join(DROPIN, "test_connection")
    _need(exe)
    r = run(exe, "-ns", ns, "-nw", nw, "-procs")
    assert r.returncode == 0, r.stderr[-2000:]


def test_process_mode_launches_back_to_back():
    """Process-mode jobs launched back to back (the launcher writes every
    role's config once, before any node starts: rewriting a role's file per
    node truncated it under a node already reading it, which then dialled the
    default scheduler port until the job hung — about once in 4-50 launches of
    test_connection -ns 2 -nw 3)."""
    exe = os.path.join(DROPIN, "test_connection")
    _need(exe)
    for i in range(40):
        r = run(exe, "-ns", 2, "-nw", 3, "-procs", timeout=30)
        assert r.returncode == 0, f"launch {i}: " + r.stderr[-2000:]


def test_dropin_simple_app_processes():
    """test_simple_app.cpp counts requests in a process-global `num` and CHECKs
    it equals 100 on every node: that holds only with one node per process."""
    exe = os.path.join(DROPIN, "test_simple_app")
    _need(exe)
    for ns, nw in [(1, 1), (2, 2)]:
        r = run(exe, "-ns", ns, "-nw", nw, "-procs")
        assert r.returncode == 0, r.stderr[-2000:]


@pytest.mark.parametrize("ns,nw", [(1, 1), (3, 2)])
def test_host_cluster_processes(ns, nw):
    exe = os.path.join(BIN, "kv_cluster_host")
    _need(exe)
    r = run(exe, "-ns", ns, "-nw", nw, "-procs")
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count(" ok") == nw


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_localpy_style_launch(tmp_path):
    """The launch protocol of tests/local.py (local.py:61-114), restated: one
    JSON config per role (PS_NUM_SERVER, PS_NUM_WORKER, PS_ROLE,
    PS_SCHEDULER_URI, PS_SCHEDULER_PORT) and one process per node started as
    `prog config log role` — no launcher of ours involved."""
    import json
    exe = os.path.join(BIN, "kv_cluster_host")
    _need(exe)
    ns, nw, port = 2, 2, _free_port()
    procs = []

    def start(role, i):
        cfg = tmp_path / f"config_{role}.json"
        cfg.write_text(json.dumps({"PS_NUM_SERVER": ns, "PS_NUM_WORKER": nw, "PS_ROLE": role,
                                   "PS_SCHEDULER_URI": "127.0.0.1", "PS_SCHEDULER_PORT": port,
                                   "PS_VERBOSE": 1}, indent=4))
        log = tmp_path / f"log_{role}{i}.txt"
        procs.append(subprocess.Popen([exe, str(cfg), str(log), role], stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))

    # local.py starts the scheduler first; start it LAST here, so the nodes
    # must wait for it
    for i in range(nw):
        start("worker", i)
    for i in range(ns):
        start("server", i)
    start("scheduler", 0)
    outs = [p.communicate(timeout=120) for p in procs]
    assert all(p.returncode == 0 for p in procs), [o[1][-1000:] for o in outs]
    assert sum(o[0].count(" ok") for o in outs) == nw


def test_process_job_fails_fast_on_a_failed_check():
    """A CHECK that fails in one process (the HBM store on a host without a GPU)
    is broadcast: every process ends, none waits on a barrier forever."""
    exe = os.path.join(DROPIN, "test_kv_app")
    _need(exe)
    if _has_gpu():
        pytest.skip("a GPU is present")
    r = run(exe, "-ns", 2, "-nw", 2, "-procs", timeout=90)
    assert r.returncode != 0
    assert "value store lives in HBM" in r.stderr


@pytest.mark.parametrize("procs", [False, True])
def test_group_broadcast(procs):
    """PostOffice::GroupBroadcast (the rendezvous ps::CreateComm hands the RCCL
    id through): every member of three groups gets its root's bytes, three
    rounds, in thread mode and through the scheduler in process mode."""
    exe = os.path.join(BIN, "comm_group")
    _need(exe)
    r = run(exe, "-ns", 2, "-nw", 3, *(["-procs"] if procs else []))
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count("bcast ok") == 6


REF_LOCAL_PY = "/root/reference/tests/local.py"


@pytest.mark.skipif(not os.path.exists(REF_LOCAL_PY), reason="reference tree absent (GPU box)")
def test_reference_local_py_launches_our_binaries(tmp_path):
    """The reference's own launcher (tests/local.py, run where the reference
    tree exists) starts our binaries unchanged: its `config log role` command
    lines select process mode.  local.py ignores its children's exit codes, so
    the check is on what the nodes print."""
    import sys
    for exe, expect in [(os.path.join(BIN, "kv_cluster_host"), 2),
                        (os.path.join(DROPIN, "test_simple_app"), 0)]:
        _need(exe)
        r = subprocess.run([sys.executable, REF_LOCAL_PY, "-ns", "2", "-nw", "2", "-exec", exe],
                           cwd=tmp_path, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        assert "Check failed" not in r.stderr and "aborted" not in r.stderr, r.stderr[-2000:]
        assert r.stdout.count(" ok") == expect, r.stdout


def test_process_job_ends_when_a_node_dies():
    """A worker process that dies without a goodbye (std::_Exit after the start
    barrier): the others see the dropped connection, abort their waits and the
    job ends non-zero within seconds instead of hanging in Finalize."""
    exe = os.path.join(BIN, "crash_node")
    _need(exe)
    r = run(exe, "-ns", 2, "-nw", 2, "-procs", timeout=60)
    assert r.returncode != 0
    assert "disconnected" in r.stderr


def test_process_mode_host_frames_travel_as_shared_memory():
    """Host frames >= 1 MiB between processes on one host are shared-memory
    mappings (internal/shm_pool.h), not socket bytes; replies that echo the
    request keys point back into the worker's own frames; /dev/shm is clean
    afterwards."""
    import re
    exe = os.path.join(BIN, "kv_cluster_host")
    _need(exe)
    r = run(exe, "-ns", 2, "-nw", 2, "-procs", 300000, env={"PS_VAN_STATS": "1"}, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count(" ok") == 2
    stats = {int(m.group(1)): (int(m.group(2)), int(m.group(3)))
             for m in re.finditer(r"van stats node (\d+): frames sent host=\d+ hbm-ipc=\d+ echoed=(\d+) shm=(\d+)",
                                  r.stderr)}
    assert stats[9][1] > 0 and stats[11][1] > 0, stats  # workers' Push frames
    assert stats[8][0] > 0 and stats[10][0] > 0, stats  # servers echo the keys back
    assert not [f for f in os.listdir("/dev/shm") if f.startswith("psg.")]


@pytest.mark.parametrize("ring", ["1", "0"])
def test_process_mode_message_ring(ring):
    """Process mode carries each connection's message bytes through a shared-
    memory ring (PS_SHM_RING=1, the default on one host) or the socket (0).
    Both run the host cluster harness with large requests whose host frames
    stay inline (PS_SHM_FRAMES=0: 300 000 keys, 2.4 MB a frame, several times
    the 1 MiB ring, so the writer waits for room as the reader drains), and the
    request round trip of the latency harness; no ring is left in /dev/shm."""
    import json
    exe = os.path.join(BIN, "kv_cluster_host")
    _need(exe)
    r = run(exe, "-ns", 2, "-nw", 2, "-procs", 300000, env={"PS_SHM_RING": ring, "PS_SHM_FRAMES": "0"},
            timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count(" ok") == 2
    lat = os.path.join(BIN, "kv_latency_host")
    _need(lat)
    r = run(lat, "-ns", 1, "-nw", 1, "-procs",
            env={"PS_SHM_RING": ring, "LAT_ITERS": "5000", "LAT_MODE": "ring" + ring}, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][0])
    assert line["iters"] == 5000 and line["us_per_request"] > 0
    print(line)
    assert not [f for f in os.listdir("/dev/shm") if f.startswith("psgring.")]


def test_process_mode_refused_ring_falls_back_to_the_socket():
    """A reader that cannot map a connection's shared-memory ring (another
    /dev/shm behind the same hostname, or no room in it) answers 'N' and the
    writer keeps every byte on the socket: the job still completes."""
    exe = os.path.join(BIN, "kv_cluster_host")
    _need(exe)
    r = run(exe, "-ns", 2, "-nw", 2, "-procs", 300000, env={"PS_SHM_RING_REFUSE": "1"}, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.count(" ok") == 2


def test_hung_process_job_prints_every_threads_stack():
    """PS_JOB_TIMEOUT_S: a process job still running at the deadline is taken
    as hung; every node prints the stacks of all its threads (SIGQUIT), then
    the launcher kills the job and exits 124.  A 3 M-key job with a 1 s limit
    stands in for a hang."""
    exe = os.path.join(BIN, "kv_cluster_host")
    _need(exe)
    e = dict(os.environ, PS_JOB_TIMEOUT_S="1")
    r = subprocess.run([exe, "-ns", "2", "-nw", "2", "-procs", "3000000"], capture_output=True, text=True,
                       timeout=60, env=e)
    assert r.returncode == 124, r.stderr[-2000:]
    assert "PS_JOB_TIMEOUT_S=1" in r.stderr
    # the scheduler, 2 servers and 2 workers each dumped, thread by thread
    assert r.stderr.count("SIGQUIT: stacks of every thread follow") == 5, r.stderr[-3000:]
    assert "RunNode" in r.stderr  # frames carry names (-rdynamic)
