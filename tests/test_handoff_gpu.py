"""A Pull reply handed out by the store's completion wait holds the request's
values (tests/harness/unit/handoff_stress.cpp).

GPUTEST_r03 caught the LR handle answering a Pull with an earlier reply's
values over a tail of the buffer (ps/lr_handle.h; the reference answers with
the post-update weights, tests/src/LRServer.h:163-177, 196-206).  The waits a
server makes before answering now rest on events (psg_store.hip,
stream_done / wait_landed) and the host copies on this runtime's own pinned
staging (src/device.cc).  Each case below runs the exact answer sequence many
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
