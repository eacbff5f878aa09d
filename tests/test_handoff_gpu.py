"""A Pull reply handed out by the store's completion wait holds the request's
values (tests/harness/unit/handoff_stress.cpp).

The waits a server makes before answering rest on events (psg_store.hip,
stream_done / wait_landed) and the host copies on this runtime's own pinned
staging (src/device.cc): a hardening step taken while GPUTEST_r03's red LR
case was open.  That case was the reference LRServer's own constructor race
(its handle installed before InitWeight, tests/src/LRServer.h:70 vs 81-87;
DESIGN.md "Parity"), not a hand-off.  Each case below runs the exact answer sequence many
times — update, Pull into one reply buffer, wait, copy out on the same stream —
and checks every element of every reply; with several threads, as in the
thread-mode cluster, each on its own stream.
"""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "_bin", "handoff_stress")


@pytest.mark.parametrize("mode", ["lr", "dense", "stretch", "keyed"])
@pytest.mark.parametrize("n,iters,threads", [(200000, 400, 1), (1000000, 200, 4)])
def test_reply_handed_out_holds_the_request_values(mode, n, iters, threads):
    if not os.path.exists(EXE):
        pytest.skip(f"{EXE} not built")
    r = subprocess.run([EXE, mode, str(n), str(iters), str(threads)], capture_output=True, text=True,
                       timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "stale_iters=0 stale_elems=0" in r.stdout, r.stdout
