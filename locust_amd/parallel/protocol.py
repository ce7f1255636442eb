"""Wire protocol between the launcher and worker daemons.

Frames are a 4-byte big-endian length followed by a UTF-8 JSON object.  Binary payloads
(spill files) travel base64-encoded in ``data``.  Every request may carry ``token``; a
daemon started with a token rejects requests without the matching one.

The reference's slave spoke raw text -- ``recv(1024)``, run ``data.split()[1:]``, reply
``ACK`` whatever happened (/root/reference/Distributor/slave.py:14-20, 30-32).  The daemon
still understands that form (see daemon.py), but answers ``NAK <rc>`` on failure.
"""
from __future__ import annotations

import json
import socket
import struct

MAX_FRAME = 256 << 20  # 256 MiB: spills are fetched in chunks below this
PROTOCOL_VERSION = 1


class ProtocolError(RuntimeError):
    pass


def send_msg(sock: socket.socket, obj: dict) -> None:
    data = json.dumps(obj, separators=(",", ":")).encode()
    if len(data) > MAX_FRAME:
        raise ProtocolError(f"frame of {len(data)} bytes exceeds {MAX_FRAME}")
    sock.sendall(struct.pack(">I", len(data)) + data)


def recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(n - len(buf), 1 << 20))
        if not chunk:
            raise ProtocolError("connection closed mid-frame")
        buf += chunk
    return bytes(buf)


def recv_msg(sock: socket.socket) -> dict:
    (n,) = struct.unpack(">I", recv_exact(sock, 4))
    if n > MAX_FRAME:
        raise ProtocolError(f"frame of {n} bytes exceeds {MAX_FRAME}")
    obj = json.loads(recv_exact(sock, n).decode())
    if not isinstance(obj, dict):
        raise ProtocolError("frame is not a JSON object")
    return obj


def request(addr: str, port: int, obj: dict, timeout: float | None = 60.0) -> dict:
    """One request/response round trip on a fresh connection."""
    with socket.create_connection((addr, port), timeout=timeout) as s:
        s.settimeout(timeout)
        send_msg(s, obj)
        return recv_msg(s)
