"""Cluster context and collectives: one process per GPU, torch.distributed over RCCL (xGMI).

Reference: the netsDB shuffle/broadcast machinery — src/communication (PDBCommunicator,
SimpleSendDataRequest), src/serverFunctionalities/source/{DispatcherServer,BroadcastServer,
HermesExecutionServer}.cc, src/queryExecution (ShuffleSink, CombinedShuffleSink,
HashPartitionedJoinBuildHTJobStage, BroadcastJoinBuildHTJobStage) which move serialized pages
between worker nodes over TCP sockets.

MI355X-native design: every worker is a rank; record batches move with collectives —
``all_to_all_single`` for hash shuffles (tensor columns stay in HBM and go straight through
RCCL), ``all_gather`` for broadcast joins, ``reduce_scatter`` for distributed aggregation of
dense blocks.  Object (host) columns are serialised into byte tensors and ride the same
collective.  ``backend='gloo'`` runs the identical code path on CPU (tests, pseudo-cluster).
"""
from __future__ import annotations

import base64
import json
import os
import time
from typing import Any, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from ..objects.nested import MapColumn, NestedColumn
from ..objects.record import RecordBatch, column_slice, lookup_type
from ..objects.strings import StringColumn
from ..storage.serde import _enc_obj, _dec_obj  # noqa: F401  (shared object codec)


class ClusterContext:
    """Rank/device information of this process (a netsDB 'worker node')."""

    def __init__(self, rank: int = 0, world_size: int = 1, device: Optional[torch.device] = None,
                 backend: Optional[str] = None, group=None, force_collectives: bool = False):
        self.rank = rank
        self.world_size = world_size
        # force_collectives: a one-rank process group (RCCL world_size 1 plus the gloo metadata group) runs the
        # multi-rank branches — streaming shuffles, partitioned joins / aggregations, all-gathers and
        # reduce-scatters on device buffers — instead of short-circuiting them (the hardware test of the RCCL
        # path on a one-GPU box; results must equal the single-process run)
        self.force_collectives = bool(force_collectives) and dist.is_initialized()
        self.device = device if device is not None else torch.device("cpu")
        self.backend = backend
        self.group = group
        # host-side metadata collectives (plan sizes, batch schemas, scalars) run on a gloo group when the
        # data backend is RCCL: a RCCL scalar all-reduce + .item() would block the host on the GPU stream
        # and stall kernel enqueueing mid-step
        self.meta_group = None
        # failure detection (utils/health.HeartbeatMonitor): every collective is issued async and waited
        # for under a watchdog that raises NodeFailure when a peer stops heartbeating, instead of hanging
        self.health = None
        self._schema_cache: Dict[int, dict] = {}
        # coll_bytes: payload bytes this rank handed to data collectives (not the gloo metadata group);
        # xgmi_pred_s: what those collectives would take on MI355X xGMI under xgmi_seconds' model
        self.stats = {"collectives": 0, "schema_cache_hits": 0, "schema_exchanges": 0, "coll_bytes": 0,
                      "xgmi_pred_s": 0.0, "data_collectives": 0}
        # single-tensor collectives (all_gather_into_tensor / reduce_scatter_tensor into one contiguous buffer):
        # RCCL's native form; gloo implements them too in this torch, so the CPU multi-rank tests run the SAME
        # branches the GPUs take. NSDB_TENSOR_COLLECTIVES=0 selects the list-based fallback (tested as well).
        env = os.environ.get("NSDB_TENSOR_COLLECTIVES")
        self.tensor_collectives = (env != "0") if env is not None else backend in ("nccl", "gloo")

    @property
    def distributed(self) -> bool:
        return self.world_size > 1 or self.force_collectives

    @staticmethod
    def from_env(device: Optional[str] = None, backend: Optional[str] = None) -> "ClusterContext":
        """torchrun-style init (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/MASTER_PORT). Rehearsal overrides:
        NSDB_DEVICE (e.g. every rank on cuda:0 of a one-GPU box) and NSDB_DIST_BACKEND (gloo: RCCL refuses two
        ranks on one GPU)."""
        ws = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        force = os.environ.get("NSDB_FORCE_COLLECTIVES", "0") == "1"
        local = int(os.environ.get("LOCAL_RANK", "0"))
        device = device or os.environ.get("NSDB_DEVICE") or None
        backend = backend or os.environ.get("NSDB_DIST_BACKEND") or None
        if device is None:
            device = f"cuda:{local}" if torch.cuda.device_count() > 0 else "cpu"
        dev = torch.device(device)
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        if (ws > 1 or force) and not dist.is_initialized():
            be = backend or ("nccl" if dev.type == "cuda" else "gloo")
            kw = {}
            if dev.type == "cuda" and be == "nccl":
                kw["device_id"] = dev
            dist.init_process_group(be, rank=rank, world_size=ws, **kw)
        be = dist.get_backend() if dist.is_initialized() else None
        ctx = ClusterContext(rank, ws, dev, be, force_collectives=force)
        ctx.attach_meta_group()
        return ctx

    def attach_meta_group(self):
        """Collective: create the gloo metadata group next to a RCCL data group."""
        if self.backend == "nccl" and self.distributed and self.meta_group is None:
            try:
                self.meta_group = dist.new_group(backend="gloo")
            except (RuntimeError, ValueError):      # no gloo transport: metadata stays on RCCL
                self.meta_group = None
        return self

    # -------------------------------------------------------------- failure-aware collective issue
    def attach_health(self, monitor):
        """Guard every collective with a heartbeat monitor (a dead rank raises NodeFailure, no hang)."""
        self.health = monitor
        return self

    def _wait(self, work):
        if work is None:
            return
        if self.health is None:
            work.wait()
            return
        while not work.is_completed():
            self.health.check()
            time.sleep(0.001)
        try:
            work.wait()
        except RuntimeError as e:
            # a transport error (peer socket reset, RCCL abort): report it as the node failure it is once
            # the heartbeats confirm which rank stopped
            deadline = time.time() + 2.5 * getattr(self.health, "timeout", 1.0)
            while time.time() < deadline:
                self.health.check()
                time.sleep(0.01)
            raise

    def _account(self, op: str, t: Optional[torch.Tensor], group=None):
        """Per-collective traffic accounting (data group only): payload bytes and the modelled xGMI time."""
        if t is None or (group is not None and group is self.meta_group):
            return
        nb = t.numel() * t.element_size()
        self.stats["data_collectives"] += 1
        self.stats["coll_bytes"] += nb
        self.stats["xgmi_pred_s"] += xgmi_seconds(op, nb, self.world_size)

    def _coll(self, fn, *args, **kw):
        """Issue a torch.distributed collective asynchronously and wait under the heartbeat watchdog."""
        self.stats["collectives"] += 1
        op = _COLL_OPS.get(fn)
        if op is not None:
            self._account(op[0], args[op[1]] if len(args) > op[1] else None, kw.get("group"))
        if self.health is not None:
            self.health.check()
            self.health.mark_progress()
        self._wait(fn(*args, async_op=True, **kw))

    # -------------------------------------------------------------- primitives
    def barrier(self):
        if self.distributed:
            if self.device.type == "cuda":
                self._coll(dist.barrier, device_ids=[self.device.index])
            else:
                self._coll(dist.barrier)

    def _comm_device(self):
        return self.device if self.backend == "nccl" else torch.device("cpu")

    def all_reduce(self, t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
        if self.distributed:
            self._coll(dist.all_reduce, t, op=op)
        return t

    def all_reduce_scalar(self, v: float, op="sum") -> float:
        if not self.distributed:
            return v
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        if self.meta_group is not None:
            t = torch.tensor([float(v)], dtype=torch.float64)
            self._coll(dist.all_reduce, t, op=rop, group=self.meta_group)
            return float(t.item())
        t = torch.tensor([float(v)], dtype=torch.float64, device=self._comm_device())
        self._coll(dist.all_reduce, t, op=rop)
        return float(t.item())

    def all_gather_ints(self, vals: Sequence[int]) -> List[List[int]]:
        """Small host-side integer metadata from every rank (sizes, ranges, schema hashes): over the gloo
        metadata group next to RCCL, so no device tensor and no host sync on the GPU stream."""
        if not self.distributed:
            return [list(vals)]
        on_meta = self.meta_group is not None
        dev = torch.device("cpu") if on_meta else self._comm_device()
        t = torch.tensor(list(vals), dtype=torch.int64, device=dev)
        outs = [torch.empty_like(t) for _ in range(self.world_size)]
        self._coll(dist.all_gather, outs, t, group=self.meta_group) if on_meta else self._coll(dist.all_gather, outs, t)
        return [o.cpu().tolist() for o in outs]

    def all_gather_tensor(self, t: torch.Tensor, sizes: Optional[Sequence[int]] = None) -> List[torch.Tensor]:
        """Variable-first-dim all_gather (rows). ``sizes`` (rows per rank) skips the size exchange when the
        caller knows them (cached plan metadata)."""
        if not self.distributed:
            return [t]
        cd = self._comm_device()
        ns = list(sizes) if sizes is not None else [x[0] for x in self.all_gather_ints([t.shape[0]])]
        mx = max(ns)
        src = t.to(cd)
        if src.shape[0] < mx:
            src = torch.cat([src, src.new_zeros((mx - src.shape[0],) + tuple(src.shape[1:]))])
        outs = [torch.empty_like(src) for _ in range(self.world_size)]
        self._coll(dist.all_gather, outs, src.contiguous())
        return [o[:k].to(t.device) for o, k in zip(outs, ns)]

    def all_to_all_rows(self, t: torch.Tensor, send_counts: Sequence[int]) -> (torch.Tensor, List[int]):
        """Rows of ``t`` (already grouped by destination) -> rows received from every rank."""
        if not self.distributed:
            return t, list(send_counts)
        cd = self._comm_device()
        recv = [row[self.rank] for row in self.all_gather_ints(list(send_counts))]   # host metadata, no sync
        src = t.to(cd).contiguous()
        out = src.new_empty((sum(recv),) + tuple(src.shape[1:]))
        if src.dtype == torch.bool:
            s8, o8 = src.view(torch.uint8), out.view(torch.uint8)
            self._coll(dist.all_to_all_single, o8, s8, recv, list(send_counts))
        else:
            self._coll(dist.all_to_all_single, out, src, recv, list(send_counts))
        return out.to(t.device), recv

    def all_to_all_bytes_async(self, out: torch.Tensor, inp: torch.Tensor, out_splits: Sequence[int],
                               in_splits: Sequence[int]):
        """Issue one variable-split all-to-all of byte buffers WITHOUT waiting (the streaming shuffle's data
        round); wait for the returned work with :meth:`_wait` (heartbeat-checked). On RCCL the transfer runs on
        the communicator's stream, ordered after the work already queued on the current stream."""
        self.stats["collectives"] += 1
        self._account("all_to_all", inp)
        if self.health is not None:
            self.health.check()
            self.health.mark_progress()
        return dist.all_to_all_single(out, inp, list(out_splits), list(in_splits), async_op=True)

    def reduce_scatter_rows(self, t: torch.Tensor, counts: Sequence[int]) -> torch.Tensor:
        """Sum ``t`` over ranks and return this rank's row slice (counts[r] rows per rank)."""
        if not self.distributed:
            return t
        cd = self._comm_device()
        if self.tensor_collectives and len(set(counts)) == 1:
            src = t.to(cd).contiguous()
            out = src.new_empty((counts[self.rank],) + tuple(t.shape[1:]))
            self._coll(dist.reduce_scatter_tensor, out, src, op=dist.ReduceOp.SUM)
            return out.to(t.device)
        full = t.to(cd).contiguous().clone()
        self._coll(dist.all_reduce, full)
        s = sum(counts[: self.rank])
        return full[s: s + counts[self.rank]].to(t.device)

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if not self.distributed:
            return obj
        if self.health is not None:
            self.health.check()
        box = [obj]
        if self.meta_group is not None:
            dist.broadcast_object_list(box, src=src, group=self.meta_group)
        else:
            dist.broadcast_object_list(box, src=src, device=self._comm_device() if self.backend == "nccl" else None)
        return box[0]

    # -------------------------------------------------------------- record batch shuffles
    def exchange(self, parts: Sequence[Optional[RecordBatch]], template: Optional[RecordBatch] = None) -> List[RecordBatch]:
        """Shuffle: ``parts[d]`` goes to rank d; returns the batches received (one per source).
        Nested columns (RecordBatch object columns, tuple key columns) are flattened for the wire."""
        ws = self.world_size
        assert len(parts) == ws
        if not self.distributed:
            return [parts[0]] if parts[0] is not None else []
        flat = [_flatten(p) if p is not None else None for p in parts]
        tflat = _flatten(template) if template is not None else None
        got = self._exchange_flat(flat, tflat)
        return [_unflatten(g) for g in got]

    def _exchange_flat(self, parts, template=None) -> List[RecordBatch]:
        ws = self.world_size
        ref = template or next((p for p in parts if p is not None), None)
        meta = _batch_meta(ref)
        ref_meta = self._agree_schema(meta)
        if ref_meta is None:
            return []
        parts = [p if p is not None else _empty_like_meta(ref_meta, self.device) for p in parts]
        counts = [p.n for p in parts]
        recv_cols: Dict[str, Any] = {}
        recv_counts = None
        # every fixed-width tensor column rides ONE all-to-all as a packed row image (one count exchange for
        # the whole batch instead of one per column); strings / nested / objects follow column by column
        from ..execution.shuffle import PackedSchema

        tcols = [cm for cm in ref_meta["columns"] if cm["kind"] == "tensor"]
        if tcols:
            ps = PackedSchema({"type": ref_meta["type"], "columns": tcols})
            t = torch.cat([ps.pack(RecordBatch({cm["name"]: _as_tensor(p.columns[cm["name"]], cm, self.device)
                                                for cm in tcols}, p.n)) for p in parts])
            out, recv_counts = self.all_to_all_rows(t, counts)
            got = ps.unpack(out)
            for cm in tcols:
                recv_cols[cm["name"]] = got.columns[cm["name"]]
        for cm in ref_meta["columns"]:
            name = cm["name"]
            if cm["kind"] == "tensor":
                continue
            if cm["kind"] == "string":
                recv_cols[name] = self._exchange_strings([p.columns[name] for p in parts], counts)
                recv_counts = recv_cols[name][1]
            elif cm["kind"] in ("nested", "map"):
                recv_cols[name], recv_counts = self._exchange_nested([p.columns[name] for p in parts], counts, cm)
            else:
                payloads = [json.dumps([_enc_plain(v) for v in p.columns[name]]).encode() for p in parts]
                data = torch.frombuffer(bytearray(b"".join(payloads)) or bytearray(b"\0"), dtype=torch.uint8)
                lens = [len(x) for x in payloads]
                if sum(lens) == 0:
                    data = data[:0]
                out, rl = self.all_to_all_rows(data, lens)
                out = out.cpu().numpy().tobytes()
                vals, off = [], 0
                for k in rl:
                    vals.append(json.loads(out[off: off + k].decode()) if k else [])
                    off += k
                recv_cols[name] = vals
        if recv_counts is None:
            recv_counts = [row[self.rank] for row in self.all_gather_ints(counts)]
        t = lookup_type(ref_meta["type"]) if ref_meta["type"] else None
        out_batches = []
        off = 0
        for src, k in enumerate(recv_counts):
            cols = {}
            for cm in ref_meta["columns"]:
                name = cm["name"]
                if cm["kind"] == "tensor":
                    cols[name] = recv_cols[name][off: off + k]
                elif cm["kind"] == "string":
                    cols[name] = recv_cols[name][0][src]
                elif cm["kind"] in ("nested", "map"):
                    cols[name] = recv_cols[name][src]
                else:
                    cols[name] = [_dec_plain(v) for v in recv_cols[name][src]]
            out_batches.append(RecordBatch(cols, k, t))
            off += k
        return out_batches

    def _agree_schema(self, meta: Optional[dict]) -> Optional[dict]:
        """Every rank learns the batch schema of the shuffle (ranks with no rows send none): a 63-bit hash
        per rank over the metadata group; the JSON schema itself travels (as a byte tensor, never pickled)
        only the first time a schema hash is seen, after that it comes from the cache."""
        import xxhash

        blob = json.dumps(meta, sort_keys=True).encode() if meta is not None else b""
        h = (xxhash.xxh64_intdigest(blob) >> 1) if meta is not None else -1
        if meta is not None:
            self._schema_cache.setdefault(h, meta)
        hs = [x[0] for x in self.all_gather_ints([h])]
        known = [x for x in hs if x >= 0]
        if not known:
            return None
        # the exchange decision must be identical on every rank: agree on "anyone missing a schema"
        missing = int(not all(x in self._schema_cache for x in known))
        if not any(x[0] for x in self.all_gather_ints([missing])):
            self.stats["schema_cache_hits"] += 1
            return self._schema_cache[known[0]]
        self.stats["schema_exchanges"] += 1
        lens = [x[0] for x in self.all_gather_ints([len(blob)])]
        mx = max(lens)
        buf = torch.zeros(mx, dtype=torch.uint8)
        if blob:
            buf[: len(blob)] = torch.frombuffer(bytearray(blob), dtype=torch.uint8)
        on_meta = self.meta_group is not None
        dev = torch.device("cpu") if on_meta else self._comm_device()
        buf = buf.to(dev)
        outs = [torch.empty_like(buf) for _ in range(self.world_size)]
        self._coll(dist.all_gather, outs, buf, group=self.meta_group) if on_meta else self._coll(dist.all_gather, outs, buf)
        got = None
        for o, n, hh in zip(outs, lens, hs):
            if hh >= 0 and n:
                m = json.loads(o[:n].cpu().numpy().tobytes().decode())
                self._schema_cache.setdefault(hh, m)
                got = got or m
        return got

    def _exchange_strings(self, cols, counts):
        """Device string columns on the wire: row lengths + packed bytes, two all-to-alls, no host
        decode. Returns (one StringColumn per source rank, received row counts)."""
        dev = self.device
        cols = [c if isinstance(c, StringColumn) else StringColumn.from_list(list(c), dev) for c in cols]
        cols = [c.to(dev) for c in cols]
        lens = torch.cat([c.offsets[1:] - c.offsets[:-1] for c in cols])
        rlens, rcounts = self.all_to_all_rows(lens, counts)
        bounds = torch.stack([torch.stack([c.offsets[0], c.offsets[-1]]) for c in cols]).cpu().tolist()   # one host read
        data = torch.cat([c.data[s:e] for c, (s, e) in zip(cols, bounds)])
        rdata, rbytes = self.all_to_all_rows(data, [e - s for s, e in bounds])
        out, ro, rb = [], 0, 0
        for k, nb in zip(rcounts, rbytes):
            offs = torch.zeros(k + 1, dtype=torch.int64, device=rlens.device)
            if k:
                torch.cumsum(rlens[ro: ro + k], 0, out=offs[1:])
            buf = torch.zeros(StringColumn._alloc_size(nb), dtype=torch.uint8, device=rdata.device)
            buf[:nb] = rdata[rb: rb + nb]
            out.append(StringColumn(buf, offs, nb))
            ro, rb = ro + k, rb + nb
        return out, rcounts

    def _exchange_nested(self, cols, counts, cm):
        """Vector / Map columns on the wire: per-row lengths in one all-to-all, then the element child
        (itself a batch, possibly nested again) shuffled recursively with per-destination element counts.
        Every rank runs the same collectives: the schema (and so this branch) was agreed beforehand."""
        dev = self.device
        cols = [_nested_rebase(c) for c in cols]
        lens = torch.cat([c.lengths().to(dev) for c in cols])
        rlens, rcounts = self.all_to_all_rows(lens, counts)
        child_parts = [_flatten(_nested_child(c)) for c in cols]
        got = self._exchange_flat(child_parts)
        out, ro = [], 0
        for src, k in enumerate(rcounts):
            offs = torch.zeros(k + 1, dtype=torch.int64, device=rlens.device)
            if k:
                torch.cumsum(rlens[ro: ro + k], 0, out=offs[1:])
            ch = _unflatten(got[src]) if got else _unflatten(_empty_like_meta(cm["child"], dev))
            out.append(MapColumn(offs, ch.columns["k"], ch.columns["v"]) if cm["kind"] == "map"
                       else NestedColumn(offs, ch.columns["v"]))
            ro += k
        return out, rcounts

    def broadcast_batch_all(self, b: Optional[RecordBatch]) -> List[RecordBatch]:
        """All-gather: every rank receives every rank's batch (broadcast join build side). Fixed-width tensor
        batches go as ONE packed row image through all_gather(_into_tensor) (one copy of the local batch on
        the wire, not world_size copies through an all-to-all); other batches use the record exchange."""
        if not self.distributed:
            return [b] if b is not None else []
        from ..execution.shuffle import PackedSchema

        flat = _flatten(b) if b is not None else None
        meta = self._agree_schema(_batch_meta(flat))
        if meta is None:
            return []
        if not PackedSchema.supports(meta):
            return self.exchange([b] * self.world_size)
        ps = PackedSchema(meta)
        if flat is not None and _batch_meta(flat) != meta:
            raise RuntimeError(f"broadcast schema mismatch: {_batch_meta(flat)} vs {meta}")
        rows = ps.pack(flat) if flat is not None else torch.empty(0, ps.row_bytes, dtype=torch.uint8, device=self.device)
        ns = [x[0] for x in self.all_gather_ints([rows.shape[0]])]
        mx = max(ns)
        if mx == 0:
            return []
        cd = self._comm_device()
        src = rows.to(cd)
        if src.shape[0] < mx:
            src = torch.cat([src, src.new_zeros((mx - src.shape[0], ps.row_bytes))])
        src = src.contiguous()
        if self.tensor_collectives:
            out = src.new_empty((self.world_size * mx, ps.row_bytes))
            self._coll(dist.all_gather_into_tensor, out, src)
            outs = [out[i * mx:(i + 1) * mx] for i in range(self.world_size)]
        else:
            outs = [torch.empty_like(src) for _ in range(self.world_size)]
            self._coll(dist.all_gather, outs, src)
        t = lookup_type(meta["type"]) if meta["type"] else None
        return [_unflatten(ps.unpack(o[:k].to(self.device), t)) for o, k in zip(outs, ns) if k]


# ---------------------------------------------------------------------------------------------- xGMI model
# MI355X node: 8 GPUs, every pair joined by one xGMI link (7 links per GPU, ~153 GB/s per link and direction), so a
# collective over the full node is bound by the bytes ONE link carries, not by a ring's slowest hop. Model (no
# congestion, alpha = fixed cost per collective):
#   all_to_all (payload P per rank): each peer link carries P / n            -> alpha + (P / n) / B
#   all_gather (P sent by each rank): every peer link carries P               -> alpha + P / B
#   reduce_scatter (P input per rank): P / n per link                         -> alpha + (P / n) / B
#   all_reduce (P per rank) = reduce_scatter + all_gather of P / n             -> 2 alpha + 2 (P / n) / B
#   broadcast (P from the root): the root's links carry P each                -> alpha + P / B
# With fewer ranks than 8 the same per-link rates hold (each rank still has a direct link to every peer).
XGMI_LINK_BPS = 153e9
XGMI_ALPHA_S = 10e-6


def xgmi_seconds(op: str, nbytes: int, world: int, link_bps: float = XGMI_LINK_BPS, alpha: float = XGMI_ALPHA_S) -> float:
    """Modelled wall time of one collective over ``world`` MI355X GPUs of one node (0 for a single rank)."""
    if world <= 1 or nbytes <= 0:
        return 0.0
    per_peer = nbytes / world
    if op == "all_reduce":
        return 2 * alpha + 2 * per_peer / link_bps
    if op in ("all_to_all", "reduce_scatter"):
        return alpha + per_peer / link_bps
    if op in ("all_gather", "broadcast"):
        return alpha + nbytes / link_bps
    return alpha


# torch.distributed functions -> (model op, index of the payload tensor among the positional arguments)
_COLL_OPS = {dist.all_reduce: ("all_reduce", 0), dist.all_gather: ("all_gather", 1),
             dist.all_gather_into_tensor: ("all_gather", 1), dist.all_to_all_single: ("all_to_all", 1),
             dist.reduce_scatter_tensor: ("reduce_scatter", 1), dist.broadcast: ("broadcast", 0)}


_SEP = "\x1f"


def _flatten(b: RecordBatch, prefix: str = "") -> RecordBatch:
    """Nested RecordBatch / tuple columns -> flat columns named prefix+SEP-paths."""
    cols = {}
    for k, c in b.columns.items():
        name = prefix + k
        if isinstance(c, RecordBatch):
            tn = c.type.type_name() if c.type is not None else ""
            inner = _flatten(c, name + _SEP + "R" + tn + _SEP)
            cols.update(inner.columns)
            if not inner.columns:
                cols[name + _SEP + "R" + tn + _SEP + "__empty__"] = torch.zeros(c.n, dtype=torch.int8)
        elif isinstance(c, tuple):
            for i, x in enumerate(c):
                cols[name + _SEP + f"T{i}"] = x
        else:
            cols[name] = c
    return RecordBatch(cols, b.n, b.type)


def _unflatten(b: RecordBatch) -> RecordBatch:
    if not any(_SEP in k for k in b.columns):
        return b
    tree: dict = {}
    for k, c in b.columns.items():
        parts = k.split(_SEP)
        node = tree
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = c

    def build(node, n, type_):
        cols = {}
        for k, v in node.items():
            if isinstance(v, dict):
                sub_keys = list(v)
                if all(s.startswith("T") and s[1:].isdigit() for s in sub_keys) and not any(
                        isinstance(x, dict) for x in v.values()):
                    cols[k] = tuple(v[f"T{i}"] for i in range(len(sub_keys)))
                else:
                    (rk,) = sub_keys
                    tn = rk[1:]
                    inner = v[rk]
                    inner.pop("__empty__", None)
                    cols[k] = build(inner, n, lookup_type(tn) if tn else None)
            else:
                cols[k] = v
        return RecordBatch(cols, n, type_)

    return build(tree, b.n, b.type)


def _batch_meta(b: Optional[RecordBatch]):
    if b is None:
        return None
    cols = []
    for k, c in b.columns.items():
        if isinstance(c, torch.Tensor):
            cols.append({"name": k, "kind": "tensor", "dtype": str(c.dtype).replace("torch.", ""),
                         "shape": list(c.shape[1:])})
        elif isinstance(c, StringColumn):
            cols.append({"name": k, "kind": "string"})
        elif isinstance(c, NestedColumn):
            cols.append({"name": k, "kind": "map" if isinstance(c, MapColumn) else "nested",
                         "child": _batch_meta(_flatten(_nested_child(_nested_rebase(c))))})
        else:
            cols.append({"name": k, "kind": "object"})
    return {"type": b.type.type_name() if b.type is not None else None, "columns": cols}


def _nested_rebase(c):
    """A nested column whose offsets start at 0 and whose children hold exactly its elements."""
    if c.offsets.numel() and int(c.offsets[0]) != 0:
        return c.slice(0, len(c))
    return c


def _nested_child(c) -> RecordBatch:
    n = int(c.offsets[-1]) if c.offsets.numel() else 0
    cols = {"v": column_slice(c.values, 0, n)}
    if isinstance(c, MapColumn):
        cols["k"] = column_slice(c.keys, 0, n)
    return RecordBatch(cols, n)


def _as_tensor(c, cm, device):
    if isinstance(c, torch.Tensor):
        return c.to(device) if c.device != device and device.type == "cuda" else c
    return torch.empty((0,) + tuple(cm["shape"]), dtype=getattr(torch, cm["dtype"]), device=device)


def _empty_like_meta(meta, device):
    cols = {}
    for cm in meta["columns"]:
        if cm["kind"] == "tensor":
            cols[cm["name"]] = torch.empty((0,) + tuple(cm["shape"]), dtype=getattr(torch, cm["dtype"]), device=device)
        elif cm["kind"] == "string":
            cols[cm["name"]] = StringColumn.empty(device)
        elif cm["kind"] in ("nested", "map"):
            ch = _unflatten(_empty_like_meta(cm["child"], device))
            off = torch.zeros(1, dtype=torch.int64, device=device)
            cols[cm["name"]] = MapColumn(off, ch.columns["k"], ch.columns["v"]) if cm["kind"] == "map" \
                else NestedColumn(off, ch.columns["v"])
        else:
            cols[cm["name"]] = []
    t = lookup_type(meta["type"]) if meta["type"] else None
    return RecordBatch(cols, 0, t)


def _enc_plain(v):
    blobs: List[bytes] = []
    if isinstance(v, torch.Tensor):
        # exact bytes + dtype + shape (a float round trip would change int64 > 2^24 and every float64)
        t = v.detach().cpu().contiguous()
        raw = t.view(torch.uint8).numpy().tobytes() if t.numel() else b""
        return {"__tt__": [base64.b64encode(raw).decode("ascii"), str(t.dtype).replace("torch.", ""),
                           list(t.shape)]}
    enc = _enc_obj(v, blobs)
    if blobs:
        raise TypeError("tensors nested in object columns cannot be shuffled; use a tensor column")
    return enc


def _dec_plain(v):
    if isinstance(v, dict) and "__tt__" in v:
        data, dt, shape = v["__tt__"]
        raw = bytearray(base64.b64decode(data))
        dtype = getattr(torch, dt)
        if not raw:
            return torch.empty(shape, dtype=dtype)
        return torch.frombuffer(raw, dtype=torch.uint8).view(dtype).reshape(shape).clone()
    return _dec_obj(v, [])


LOCAL = ClusterContext()

__all__ = ["ClusterContext", "LOCAL", "xgmi_seconds"]
