"""Concurrent jobs on separate HIP streams.

The reference's master (src/serverFunctionalities/source/QuerySchedulerServer.cc) schedules the
stages of independent jobs onto the worker pool so that they can run at the same time.  On one
MI355X the equivalent is a second hardware queue: an independent job (e.g. the conv2d block next to
the FF-NN jobs of bench.py) is enqueued on its own HIP stream, so its kernels fill the CUs that the
main job's short/under-filled kernels leave idle (split-K reduce, the 228-tile output-layer GEMM,
row softmax) instead of queueing behind them.

Ordering contract:
  * ``submit(fn)`` by default makes the job stream wait for everything already enqueued on the
    caller's stream (the job may read data produced there).  ``independent=True`` skips that wait:
    the caller declares the job's inputs resident and not written by in-flight work.
  * ``JobHandle.wait()`` makes the caller's current stream wait for the job (stream-ordered, no host
    sync); ``JobHandle.synchronize()`` blocks the host.
  * Buffers a job allocates belong to its stream in the caching allocator.  A consumer on another
    stream must ``wait()`` first; when such buffers are then freed by a later job on the same job
    stream, ``submit`` of that later job orders it after the consumer by default (drop
    ``independent`` for jobs that replace outputs another stream has read).
On CPU every job runs inline and handles are already complete.

"""
from __future__ import annotations

import threading
from typing import Callable, Dict, List, Optional, Tuple

import torch

_armed_lock = threading.Lock()


def _stream_key(device) -> Tuple[int, int]:
    dev = torch.device(device)
    return (dev.index or 0, torch.cuda.current_stream(dev).cuda_stream)


# operand prefetches armed per (device, stream): ops.gemm_nt hands the tensor to the first long 8-phase GEMM enqueued
# on THAT stream, whose workgroups read it into the Infinity Cache as they finish (gemm.hip GemmParams::pf_ptr)
_armed_pf: Dict[Tuple[int, int], torch.Tensor] = {}


def arm_operand_prefetch(tensor: torch.Tensor):
    """Arm ``tensor`` (a later kernel's operand on the current stream) for the next long GEMM on this stream."""
    if not isinstance(tensor, torch.Tensor) or not tensor.is_cuda:
        return False
    with _armed_lock:
        _armed_pf[_stream_key(tensor.device)] = tensor
    return True


def disarm_operand_prefetch(device):
    if _armed_pf and torch.device(device).type == "cuda":
        with _armed_lock:
            _armed_pf.pop(_stream_key(device), None)


def take_operand_prefetch(device) -> Optional[torch.Tensor]:
    """The operand prefetch armed on the current stream of ``device`` (removed: one launch takes it)."""
    if not _armed_pf or torch.device(device).type != "cuda":
        return None
    with _armed_lock:
        return _armed_pf.pop(_stream_key(device), None)


class JobHandle:
    def __init__(self, result, event: Optional["torch.cuda.Event"], stream: Optional["torch.cuda.Stream"],
                 device=None):
        self.result = result
        self.device = device
        self.event = event
        self.stream = stream

    def wait(self, stream: Optional["torch.cuda.Stream"] = None):
        """Stream-ordered join: ``stream`` (default: current) waits for the job's kernels."""
        if self.event is not None:
            (stream or torch.cuda.current_stream(self.device)).wait_event(self.event)
        return self.result

    def done(self) -> bool:
        return self.event is None or self.event.query()

    def synchronize(self):
        if self.event is not None:
            self.event.synchronize()
        return self.result


class JobStreams:
    """A small pool of HIP streams for concurrently executing independent jobs on one device.

    ``lanes`` streams are created lazily; jobs submitted with the same ``lane`` are serialised on
    that stream (a lane is an in-order job queue, like one reference worker's job queue)."""

    def __init__(self, device, lanes: int = 2, priority: int = 0, lane_priority: Optional[dict] = None):
        self.device = torch.device(device)
        self.lanes = max(1, int(lanes))
        self.priority = priority
        self.lane_priority = dict(lane_priority or {})
        self._streams: List[Optional[torch.cuda.Stream]] = [None] * self.lanes
        self.submitted = 0

    @property
    def on_gpu(self) -> bool:
        return self.device.type == "cuda"

    def stream(self, lane: int = 0) -> "torch.cuda.Stream":
        lane %= self.lanes
        if self._streams[lane] is None:
            self._streams[lane] = torch.cuda.Stream(self.device, priority=self.lane_priority.get(lane, self.priority))
        return self._streams[lane]

    def submit(self, fn: Callable, *args, lane: int = 0, independent: bool = False, **kwargs) -> JobHandle:
        self.submitted += 1
        if not self.on_gpu:
            return JobHandle(fn(*args, **kwargs), None, None)
        s = self.stream(lane)
        caller = torch.cuda.current_stream(self.device)
        if not independent:
            s.wait_stream(caller)
        with torch.cuda.stream(s):
            res = fn(*args, **kwargs)
            ev = torch.cuda.Event()
            ev.record(s)
        return JobHandle(res, ev, s, self.device)

    def wait_all(self, stream: Optional["torch.cuda.Stream"] = None):
        """Caller's stream waits for every lane (stream-ordered barrier over all submitted jobs)."""
        if not self.on_gpu:
            return
        cur = stream or torch.cuda.current_stream(self.device)
        for s in self._streams:
            if s is not None:
                cur.wait_stream(s)
