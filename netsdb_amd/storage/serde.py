"""Page serialisation: RecordBatch <-> bytes (the on-page / on-disk / on-wire format).

Reference: pages hold raw PDB object graphs (src/storage/headers/PDBPage.h; objects are made
relocatable by offset Handles).  Here a page image is:

    [8-byte header length][JSON header][column payloads, 64-byte aligned]

numeric/tensor columns are raw little-endian buffers; object columns are JSON with typed
encodings for PDBObjects and tensors.  Nothing is ever unpickled.
"""
from __future__ import annotations

import json
import struct
from typing import Any, Dict, List

import numpy as np
import torch

from ..objects.record import PDBObject, RecordBatch, lookup_type
from ..objects.nested import MapColumn, NestedColumn
from ..objects.strings import StringColumn

_ALIGN = 64
_DT = {torch.float32: "f32", torch.float64: "f64", torch.float16: "f16", torch.bfloat16: "bf16", torch.int64: "i64",
       torch.int32: "i32", torch.int16: "i16", torch.int8: "i8", torch.uint8: "u8", torch.bool: "bool"}
_DT_INV = {v: k for k, v in _DT.items()}


def _tensor_bytes(t: torch.Tensor) -> bytes:
    t = t.detach().contiguous().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().tobytes()
    return t.numpy().tobytes()


def _tensor_from(buf: memoryview, dtype: str, shape) -> torch.Tensor:
    dt = _DT_INV[dtype]
    if dt == torch.bfloat16:
        arr = np.frombuffer(buf, dtype=np.int16).copy()
        return torch.from_numpy(arr).view(torch.bfloat16).reshape(shape)
    npdt = torch.empty(0, dtype=dt).numpy().dtype
    arr = np.frombuffer(buf, dtype=npdt).copy()
    return torch.from_numpy(arr).reshape(shape)


def _enc_obj(v: Any, blobs: List[bytes]):
    if v is None or isinstance(v, (bool, int, float, str)):
        return v
    if isinstance(v, torch.Tensor):
        blobs.append(_tensor_bytes(v))
        return {"__t__": [len(blobs) - 1, _DT[v.dtype], list(v.shape)]}
    if isinstance(v, PDBObject):
        return {"__o__": v.type_name(), "f": {k: _enc_obj(x, blobs) for k, x in v.to_dict().items()}}
    if isinstance(v, (list, tuple)):
        return {"__l__": [_enc_obj(x, blobs) for x in v], "tuple": isinstance(v, tuple)}
    if isinstance(v, dict):
        return {"__d__": [[_enc_obj(k, blobs), _enc_obj(x, blobs)] for k, x in v.items()]}
    if isinstance(v, (np.integer, np.floating)):
        return v.item()
    raise TypeError(f"cannot serialise object of type {type(v)}")


def _dec_obj(v: Any, blobs: List[torch.Tensor]):
    if isinstance(v, dict):
        if "__t__" in v:
            return blobs[v["__t__"][0]]
        if "__o__" in v:
            cls = lookup_type(v["__o__"])
            o = cls.__new__(cls)
            for k, x in v["f"].items():
                setattr(o, k, _dec_obj(x, blobs))
            return o
        if "__l__" in v:
            lst = [_dec_obj(x, blobs) for x in v["__l__"]]
            return tuple(lst) if v.get("tuple") else lst
        if "__d__" in v:
            return {_dec_obj(k, blobs): _dec_obj(x, blobs) for k, x in v["__d__"]}
    return v


def serialize_batch(batch: RecordBatch) -> bytes:
    cols_meta = []
    payloads: List[bytes] = []
    off = 0

    def add(b: bytes) -> int:
        nonlocal off
        start = off
        payloads.append(b)
        pad = (-len(b)) % _ALIGN
        if pad:
            payloads.append(b"\0" * pad)
        off += len(b) + pad
        return start

    for name, c in batch.columns.items():
        if isinstance(c, torch.Tensor):
            b = _tensor_bytes(c)
            cols_meta.append({"name": name, "kind": "tensor", "dtype": _DT[c.dtype], "shape": list(c.shape),
                              "off": add(b), "len": len(b)})
        elif isinstance(c, NestedColumn):       # Vector / Map field: offsets + element (and key) children
            if c.offsets.numel() and int(c.offsets[0]) != 0:
                c = c.slice(0, len(c))
            ob = _tensor_bytes(c.offsets.cpu() - c.offsets[0].cpu())
            ch = {"v": c.values}
            if isinstance(c, MapColumn):
                ch["k"] = c.keys
            b = serialize_batch(RecordBatch(ch, int(c.offsets[-1] - c.offsets[0]) if c.offsets.numel() else 0))
            cols_meta.append({"name": name, "kind": "map" if isinstance(c, MapColumn) else "nested",
                              "n": c.offsets.numel() - 1, "off": add(ob), "len": len(ob), "boff": add(b),
                              "blen": len(b)})
        elif isinstance(c, RecordBatch):        # nested record column (an engine tuple set's object column)
            b = serialize_batch(c)
            cols_meta.append({"name": name, "kind": "batch", "off": add(b), "len": len(b)})
        elif isinstance(c, tuple):              # tuple column (multi-attribute keys): a nested batch of its parts
            b = serialize_batch(RecordBatch({f"t{i}": x for i, x in enumerate(c)}, batch.n))
            cols_meta.append({"name": name, "kind": "tuple", "k": len(c), "off": add(b), "len": len(b)})
        elif isinstance(c, StringColumn):       # packed UTF-8 + offsets: no per-string JSON
            o = c.offsets.cpu()
            base = int(o[0]) if o.numel() else 0
            ob = _tensor_bytes(o - base)
            db = c.data[base: base + int(o[-1]) - base].cpu().numpy().tobytes() if o.numel() > 1 else b""
            cols_meta.append({"name": name, "kind": "string", "n": o.numel() - 1, "off": add(ob), "len": len(ob),
                              "doff": add(db), "dlen": len(db)})
        else:
            blobs: List[bytes] = []
            enc = [_enc_obj(v, blobs) for v in c]
            js = json.dumps(enc).encode()
            blob_meta = []
            for bb in blobs:
                blob_meta.append([add(bb), len(bb)])
            cols_meta.append({"name": name, "kind": "object", "off": add(js), "len": len(js), "blobs": blob_meta})
    # blob dtypes are inside the JSON; store them flat
    header = {"type": batch.type.type_name() if batch.type is not None else None, "n": batch.n, "columns": cols_meta}
    hb = json.dumps(header).encode()
    return struct.pack("<Q", len(hb)) + hb + b"".join(payloads)


def deserialize_batch(data) -> RecordBatch:
    mv = memoryview(data)
    (hl,) = struct.unpack("<Q", mv[:8])
    header = json.loads(bytes(mv[8:8 + hl]).decode())
    base = 8 + hl
    cols: Dict[str, Any] = {}
    for cm in header["columns"]:
        seg = mv[base + cm["off"]: base + cm["off"] + cm["len"]]
        if cm["kind"] == "tensor":
            cols[cm["name"]] = _tensor_from(seg, cm["dtype"], cm["shape"])
        elif cm["kind"] == "batch":
            cols[cm["name"]] = deserialize_batch(seg)
        elif cm["kind"] in ("nested", "map"):
            offs = _tensor_from(seg, "i64", [cm["n"] + 1])
            inner = deserialize_batch(mv[base + cm["boff"]: base + cm["boff"] + cm["blen"]])
            cols[cm["name"]] = (MapColumn(offs, inner.columns["k"], inner.columns["v"]) if cm["kind"] == "map"
                                else NestedColumn(offs, inner.columns["v"]))
        elif cm["kind"] == "tuple":
            inner = deserialize_batch(seg)
            cols[cm["name"]] = tuple(inner.columns[f"t{i}"] for i in range(cm["k"]))
        elif cm["kind"] == "string":
            offs = _tensor_from(seg, "i64", [cm["n"] + 1])
            raw = np.frombuffer(mv[base + cm["doff"]: base + cm["doff"] + cm["dlen"]], dtype=np.uint8)
            buf = np.zeros(StringColumn._alloc_size(cm["dlen"]), dtype=np.uint8)
            buf[: cm["dlen"]] = raw
            cols[cm["name"]] = StringColumn(torch.from_numpy(buf), offs, cm["dlen"])
        else:
            enc = json.loads(bytes(seg).decode())
            raw_blobs = [mv[base + o: base + o + ln] for o, ln in cm.get("blobs", [])]
            # resolve tensor blobs lazily using the dtype/shape recorded at the use site
            blobs_t: List[torch.Tensor] = [None] * len(raw_blobs)  # type: ignore[list-item]

            def fix(v):
                if isinstance(v, dict):
                    if "__t__" in v:
                        i, dt, sh = v["__t__"]
                        if blobs_t[i] is None:
                            blobs_t[i] = _tensor_from(raw_blobs[i], dt, sh)
                        return {"__t__": [i]}
                    return {k: (fix(x) if k != "__o__" else x) for k, x in v.items()}
                if isinstance(v, list):
                    return [fix(x) for x in v]
                return v

            enc = fix(enc)
            cols[cm["name"]] = [_dec_obj(v, blobs_t) for v in enc]
    t = lookup_type(header["type"]) if header["type"] else None
    return RecordBatch(cols, header["n"], t)


__all__ = ["serialize_batch", "deserialize_batch"]
