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

Tail-gated jobs (``TailTrigger``): a long split-K GEMM (the FF layer-1 product) runs as ONE resident wave of
256 workgroups whose finish times spread over tens of microseconds (XCD rate differences and stragglers,
profiles/r2_gemm1_study) — CUs that finish first sit idle until the launch drains. An independent job submitted
with ``start_on=trigger.arm()`` (armed BEFORE the GEMM is enqueued) is held on its stream by the GPU command
processor (hipStreamWaitValue32) until the first workgroup of that GEMM finishes its main loop, so its kernels
fill exactly those idle CUs: it can neither start early and take CUs the GEMM's wave needs, nor wait for
the GEMM's whole tail.
"""
from __future__ import annotations

import threading
from typing import Callable, Dict, List, Optional, Tuple

import torch

# tail triggers armed per (device, stream): ops.gemm_nt hands the trigger to the first eligible GEMM enqueued on
# THAT stream (no process-wide state in the kernel library; GEMMs on other streams never take it)
_armed: Dict[Tuple[int, int], "TailTrigger"] = {}
_armed_lock = threading.Lock()


def _stream_key(device) -> Tuple[int, int]:
    dev = torch.device(device)
    return (dev.index or 0, torch.cuda.current_stream(dev).cuda_stream)


def armed_trigger(device) -> Optional["TailTrigger"]:
    """The tail trigger armed on the current stream of ``device``, if any (ops.gemm_nt's per-call lookup)."""
    if not _armed or torch.device(device).type != "cuda":
        return None
    with _armed_lock:
        return _armed.get(_stream_key(device))


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


class TailTrigger:
    """Device flag raised by the workgroups of the next long 8-phase GEMM launch enqueued on the stream that
    armed it (see module doc).

    ``mode="start"`` (a START gate, :meth:`PDBClient.arm_start_gate`): the launch that takes it leaves
    ``reserve_cus`` CUs free (fewer split-K slices: the layer-1 GEMM is power-limited, so 240 instead of 256
    workgroups cost it ~2 %), every workgroup adds 1 to the flag when it starts, and the gated job waits for
    flag >= base + workgroups — it is dispatched only once the whole GEMM holds its CUs, so it runs on exactly
    the reserved ones, beside the GEMM, instead of in its tail.

    ``arm()`` (on the stream that will run the GEMM) before enqueuing the job whose GEMM tail should be filled;
    ``JobStreams.submit(..., start_on=trigger)`` then gates the submitted job on it. The gate is only installed
    when a launch actually took the armed trigger (every workgroup of that launch writes the flag, so the wait
    always ends); otherwise the job starts ungated. Arming is per stream: a GEMM enqueued on another stream
    (another job lane, another thread's stream) never takes it."""

    def __init__(self, device, mode: str = "tail", reserve_cus: int = 0):
        if mode not in ("tail", "start"):
            raise ValueError(f"trigger mode {mode!r}: 'tail' or 'start'")
        self.mode = mode
        self.reserve_cus = int(reserve_cus)
        self.count = 0       # start mode: workgroups counted into the flag so far (the gate's wait value)
        self.device = torch.device(device)
        self.flag = torch.zeros(1, dtype=torch.int32, device=self.device) if self.device.type == "cuda" else None
        if self.flag is not None:
            # the command processor may evaluate a gate on another stream before a stream-ordered zero-fill has
            # run: a recycled allocation still holding a stale value >= the first epoch would open the gate early
            torch.cuda.synchronize(self.device)
        self.epoch = 0
        self.armed = False
        self.consumed = False
        self._key = None
        self.gated = 0       # jobs that were actually gated (stats / tests)

    def arm(self) -> "TailTrigger":
        if self.flag is None:
            return self
        from .. import _ext

        self.epoch = self.epoch % 0x7FFFFFFF + 1     # flag values only grow (atomic max), never wrap to 0
        if (self.epoch == 1 and self.gated) or self.count > 0x7FFF0000:   # wrapped: restart from a zero flag
            torch.cuda.synchronize(self.device)
            self.flag.zero_()
            torch.cuda.synchronize(self.device)
            self.count = 0
        _ext.hip()                                   # the GEMM that takes it runs on the HIP kernels
        self.disarm()
        self._key = _stream_key(self.device)
        with _armed_lock:
            _armed[self._key] = self
        self.armed = True
        self.consumed = False
        return self

    def take(self, workgroups: int = 0) -> Tuple[torch.Tensor, int]:
        """Called by the GEMM launch that takes the trigger: (flag, value) for that launch only (start mode: the
        launch's ``workgroups`` each add 1; the value is the flag once all have started)."""
        self.consumed = True
        self.disarm()
        if self.mode == "start":
            self.count += int(workgroups)
            return self.flag, self.count
        return self.flag, self.epoch

    def untake(self, workgroups: int = 0):
        """The launch that took the trigger failed to enqueue: nothing will raise the flag, so no job may be gated
        on it (a gate on a value that never comes would stall its stream forever)."""
        self.consumed = False
        if self.mode == "start":
            self.count -= int(workgroups)

    def disarm(self):
        with _armed_lock:
            if self._key is not None and _armed.get(self._key) is self:
                del _armed[self._key]
        self._key = None

    def gate(self, stream) -> bool:
        """Make ``stream`` wait on the GPU for the armed launch's first finished workgroup."""
        if not self.armed or self.flag is None:
            return False
        from .. import _ext

        h = _ext.hip()
        self.armed = False
        if not self.consumed:
            self.disarm()
            return False
        self.consumed = False
        with torch.cuda.stream(stream):
            h.stream_wait_value(self.flag, self.count if self.mode == "start" else self.epoch)
        self.gated += 1
        return True


class TailPrefetch:
    """Read a later kernel's operands into the Infinity Cache during a long GEMM's ragged tail.

    The FF layer-1 GEMM streams 2.4 GB through the cache, so the output layer's 29 MB weight arrives from HBM
    (the output GEMM runs ~20 us slower in the bench than cache-hot). ``begin(tensors)`` arms a
    :class:`TailTrigger` on the current stream; the next long 8-phase GEMM enqueued there takes it.
    ``launched()`` (after that GEMM was enqueued) gates a low-priority side stream on the trigger and enqueues
    ``ops.prefetch`` of the tensors there: it starts when the GEMM's first workgroup finishes, on the CUs the
    tail leaves idle. ``end()`` makes the current stream wait for the side stream (call it after the consumer
    was enqueued, so the consumer never waits for the prefetch). Nothing happens when no launch took the
    trigger, on CPU tensors or during graph capture.

    Measured (profiles/r3_s2): a cold output GEMM call takes 71.6 us, 65.7 after an explicit prefetch, 54.7 when
    its operands are still in the XCDs' L2s from the previous call — the prefetch warms the Infinity Cache but
    not the L2 of the XCD whose tiles read each panel; in the bench the gated prefetch costs more than it saves
    (1.021 vs 0.992 ms per step), so the engine option is off by default."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.trigger = TailTrigger(self.device)
        self.stream = None
        self._tensors = None
        self._event = None
        self.prefetches = 0

    def begin(self, tensors) -> bool:
        self._tensors, self._event = None, None
        if self.device.type != "cuda" or torch.cuda.is_current_stream_capturing():
            return False
        self._tensors = [t for t in tensors if isinstance(t, torch.Tensor) and t.is_cuda]
        if not self._tensors:
            return False
        if self.stream is None:
            lo, _ = torch.cuda.Stream.priority_range()
            self.stream = torch.cuda.Stream(self.device, priority=lo)
        # the tensors' producers so far (stream order); recorded BEFORE the GEMM is enqueued, so the side stream
        # does not wait for the GEMM itself — only for its first finished workgroup (the gate)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        self.trigger.arm()
        return True

    def launched(self):
        if not self._tensors:
            return
        from .. import ops

        if not self.trigger.gate(self.stream):
            self._tensors = None
            return
        with torch.cuda.stream(self.stream):
            ops.prefetch(self._tensors)
            self._event = torch.cuda.Event()
            self._event.record(self.stream)
        for t in self._tensors:
            t.record_stream(self.stream)
        self._tensors = None
        self.prefetches += 1

    def end(self):
        self.trigger.disarm()
        if self._event is not None:
            torch.cuda.current_stream(self.device).wait_event(self._event)
            self._event = None


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

    def submit(self, fn: Callable, *args, lane: int = 0, independent: bool = False,
               start_on: Optional[TailTrigger] = None, **kwargs) -> JobHandle:
        self.submitted += 1
        if not self.on_gpu:
            return JobHandle(fn(*args, **kwargs), None, None)
        s = self.stream(lane)
        caller = torch.cuda.current_stream(self.device)
        if not independent:
            s.wait_stream(caller)
        if start_on is not None:
            start_on.gate(s)
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
