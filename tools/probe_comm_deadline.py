"""Diagnose psg_comm_init's rendezvous deadline: a world-2 communicator whose
rank 1 never joins.  Prints where the time goes (PSG_COMM_DEBUG=1)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "parameter-server_amd", "python"))
import psg  # noqa: E402

psg.set_device(0)
uid = psg.comm_id()
t0 = time.monotonic()
try:
    psg.Comm(uid, 2, 0)
    print("JOINED", flush=True)
except psg.PsgError as e:
    print("FAILED", e.code, round(time.monotonic() - t0, 2), str(e), flush=True)
print("exiting", round(time.monotonic() - t0, 2), flush=True)
