"""Rank rendezvous for one node without torch: a star of TCP sockets on loopback.

bench.py's N > 1 job needs only a handful of host-side group operations — hand
the RCCL unique id and the hipIpc handles around, barriers around the timed
region, a max over ranks of the step times.  The reference bootstraps its own
node group the same way, without a framework: every node connects to the
scheduler, which answers ADD_NODE and BARRIER (src/internal/Van.cpp:187-220,
:320-442).  Here rank 0 plays the scheduler's part.

Doing this without torch.distributed keeps torch (and its bundled
libamdhip64 / librccl of another ROCm release) out of the bench process, so
libpsgpu.so runs on /opt/rocm's HIP and RCCL at every N.

Rendezvous: rank 0 listens on an ephemeral loopback port and publishes it in a
file named after the launcher (parent pid) and MASTER_PORT; the other ranks
read the file and connect.  Messages are length-prefixed pickles between the
job's own processes.
"""
from __future__ import annotations

import os
import pickle
import socket
import struct
import tempfile
import time

_HDR = struct.Struct("<Q")


def _send(sock: socket.socket, obj) -> None:
    b = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
    sock.sendall(_HDR.pack(len(b)) + b)


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(n - len(buf), 1 << 20))
        if not chunk:
            raise ConnectionError("psg_group: peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock: socket.socket):
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    return pickle.loads(_recv_exact(sock, n))


def default_rendezvous_file() -> str:
    """One name per job: the launcher's pid (torch.distributed.run, or the
    test's parent process) and MASTER_PORT; PSG_RDZV_FILE overrides it."""
    f = os.environ.get("PSG_RDZV_FILE")
    if f:
        return f
    port = os.environ.get("MASTER_PORT", "0")
    return os.path.join(tempfile.gettempdir(), f"psg_rdzv_{os.getuid()}_{os.getppid()}_{port}")


class SocketGroup:
    """barrier / broadcast / all_gather / allreduce_max over a loopback star."""

    def __init__(self, rank: int, world: int, path: str | None = None, timeout_s: float | None = None):
        # every rendezvous and every later collective waits at most timeout_s
        # (PSG_GROUP_TIMEOUT_S, default 180 s) for a peer, then raises: a rank
        # that died or hangs ends the job with an error instead of a hang
        if timeout_s is None:
            timeout_s = float(os.environ.get("PSG_GROUP_TIMEOUT_S", "180"))
        self.rank, self.world = rank, world
        self.path = path or default_rendezvous_file()
        self.peers: list[socket.socket] = []
        self.sock = None
        self._listen = None
        if world == 1:
            return
        deadline = time.monotonic() + timeout_s
        if rank == 0:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass
            ls = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            ls.bind(("127.0.0.1", 0))
            ls.listen(world)
            self._listen = ls
            tmp = f"{self.path}.{os.getpid()}.tmp"
            with open(tmp, "w") as f:
                f.write(str(ls.getsockname()[1]))
            os.replace(tmp, self.path)
            got: dict[int, socket.socket] = {}
            ls.settimeout(1.0)
            while len(got) < world - 1:
                if time.monotonic() > deadline:
                    raise TimeoutError(f"psg_group: {len(got) + 1} of {world} ranks joined")
                try:
                    c, _ = ls.accept()
                except socket.timeout:
                    continue
                c.settimeout(timeout_s)
                hello = _recv(c)
                if not (isinstance(hello, tuple) and len(hello) == 2 and hello[1] == world
                        and 0 < hello[0] < world and hello[0] not in got):
                    c.close()  # a stale client of another job
                    continue
                c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                got[hello[0]] = c
            self.peers = [got[r] for r in range(1, world)]
            for c in self.peers:
                _send(c, "ok")
        else:
            while True:
                if time.monotonic() > deadline:
                    raise TimeoutError(f"psg_group: rank {rank} found no rank 0 at {self.path}")
                try:
                    with open(self.path) as f:
                        port = int(f.read().strip())
                    c = socket.create_connection(("127.0.0.1", port), timeout=5.0)
                    c.settimeout(timeout_s)
                    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    _send(c, (rank, world))
                    if _recv(c) == "ok":
                        self.sock = c
                        break
                    c.close()
                except (OSError, ValueError, ConnectionError, EOFError):
                    time.sleep(0.05)

    # -- collectives (rank order everywhere) ------------------------------------
    def all_gather(self, obj) -> list:
        if self.world == 1:
            return [obj]
        if self.rank == 0:
            out = [obj] + [_recv(c) for c in self.peers]
            for c in self.peers:
                _send(c, out)
            return out
        _send(self.sock, obj)
        return _recv(self.sock)

    def broadcast(self, obj=None, src: int = 0):
        return self.all_gather(obj if self.rank == src else None)[src]

    def barrier(self) -> None:
        self.all_gather(None)

    def allreduce_max(self, xs):
        rows = self.all_gather(list(xs))
        return [max(r[i] for r in rows) for i in range(len(rows[0]))]

    def close(self) -> None:
        try:
            self.barrier()  # nobody leaves while a peer still talks to it
        except Exception:  # noqa: BLE001
            pass
        for c in self.peers:
            c.close()
        if self.sock is not None:
            self.sock.close()
        if self._listen is not None:
            self._listen.close()
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass
        self.peers, self.sock, self._listen = [], None, None


class TorchGroup:
    """The same interface over an initialised torch.distributed process group
    (the CPU gloo rehearsal in tests/test_dist.py)."""

    def __init__(self, dist):
        self.dist = dist
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def all_gather(self, obj) -> list:
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def broadcast(self, obj=None, src: int = 0):
        box = [obj if self.rank == src else None]
        self.dist.broadcast_object_list(box, src=src)
        return box[0]

    def barrier(self) -> None:
        self.dist.barrier()

    def allreduce_max(self, xs):
        rows = self.all_gather(list(xs))
        return [max(r[i] for r in rows) for i in range(len(rows[0]))]

    def close(self) -> None:
        pass
