"""Length-prefixed JSON framing + typed encoding of tensors / PDB objects (no pickle)."""
from __future__ import annotations

import base64
import json
import socket
import struct

import numpy as np
import torch

from ..objects.record import PDBObject, lookup_type

_MAX = 1 << 31


def encode(v):
    if isinstance(v, torch.Tensor):
        t = v.detach().cpu()
        dt = str(t.dtype).replace("torch.", "")
        if t.dtype == torch.bfloat16:
            raw = t.contiguous().view(torch.int16).numpy().tobytes()
        else:
            raw = t.contiguous().numpy().tobytes()
        return {"__tensor__": [dt, list(t.shape), base64.b64encode(raw).decode()]}
    if isinstance(v, PDBObject):
        return {"__obj__": v.type_name(), "f": {k: encode(x) for k, x in v.to_dict().items()}}
    if isinstance(v, dict):
        return {"__dict__": [[encode(k), encode(x)] for k, x in v.items()]}
    if isinstance(v, (list, tuple)):
        return [encode(x) for x in v]
    if isinstance(v, (np.integer, np.floating)):
        return v.item()
    return v


def decode(v):
    if isinstance(v, dict):
        if "__tensor__" in v:
            dt, shape, b64 = v["__tensor__"]
            raw = base64.b64decode(b64)
            if dt == "bfloat16":
                return torch.from_numpy(np.frombuffer(raw, dtype=np.int16).copy()).view(torch.bfloat16).reshape(shape)
            npdt = torch.empty(0, dtype=getattr(torch, dt)).numpy().dtype
            return torch.from_numpy(np.frombuffer(raw, dtype=npdt).copy()).reshape(shape)
        if "__obj__" in v:
            cls = lookup_type(v["__obj__"])
            o = cls.__new__(cls)
            for k, x in v["f"].items():
                setattr(o, k, decode(x))
            return o
        if "__dict__" in v:
            return {decode(k): decode(x) for k, x in v["__dict__"]}
        return {k: decode(x) for k, x in v.items()}
    if isinstance(v, list):
        return [decode(x) for x in v]
    return v


def send_msg(sock: socket.socket, obj) -> None:
    data = json.dumps(encode(obj)).encode()
    sock.sendall(struct.pack(">I", len(data)) + data)


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(min(1 << 20, n - len(buf)))
        if not chunk:
            raise ConnectionError("peer closed the connection")
        buf += chunk
    return bytes(buf)


def recv_msg(sock: socket.socket):
    (n,) = struct.unpack(">I", _recv_exact(sock, 4))
    if n >= _MAX:
        raise ValueError("message too large")
    return decode(json.loads(_recv_exact(sock, n).decode()))


__all__ = ["encode", "decode", "send_msg", "recv_msg"]
