"""torch view of the streaming continuity object (include/gsdr/stream.h).

    s = Stream("fm", taps, decimation=4, rf_sample_rate=1e6, channel_frequency=1e5,
               frequency_deviation=2e4)
    for chunk in chunks:            # complex64 (or int8 I/Q) device tensors of any length
        audio = s.process(chunk)    # every output that became computable, in order

Concatenated over the calls, the outputs equal one gsdrFirFC / gsdrFmDemod / gsdrAmDemod call over
the concatenated input, bit for bit.

A list of channel frequencies (and, for FM, of deviations) makes a multi-channel stream
(gsdrxStreamCreateMulti): process() then returns a (channels, outputs) tensor whose row c is the
single-channel stream of channel c, bit for bit.
"""
from __future__ import annotations

import ctypes

import torch

from .abi import GsdrError, check, lib
from .ops import stream_of

KINDS = {"fir": 0, "fm": 1, "am": 2}


class Stream:
    def __init__(self, kind: str, taps: torch.Tensor, decimation: int, rf_sample_rate: float = 1.0,
                 tuning_frequency: float = 0.0, channel_frequency: float = 0.0, frequency_deviation: float = 1.0,
                 first_sample_index: int = 0, int8: bool = False):
        if kind not in KINDS:
            raise ValueError(f"kind must be one of {sorted(KINDS)}")
        if taps.dtype != torch.float32 or taps.device.type != "cuda" or not taps.is_contiguous():
            raise TypeError("taps must be a contiguous float32 device tensor")
        self.kind, self.int8, self.taps = kind, int8, taps  # keep taps alive: the stream reads them
        self.device = taps.device
        self._h = ctypes.c_void_p()
        self.channels = None  # single-channel stream
        if isinstance(channel_frequency, (list, tuple)):
            C = len(channel_frequency)
            devs = frequency_deviation if isinstance(frequency_deviation, (list, tuple)) else [frequency_deviation] * C
            if len(devs) != C:
                raise ValueError("one frequency deviation per channel")
            self.channels = C
            chans = (ctypes.c_float * C)(*[float(f) for f in channel_frequency])
            dv = (ctypes.c_float * C)(*[float(d) for d in devs])
            check("gsdrxStreamCreateMulti", lib.gsdrxStreamCreateMulti(
                ctypes.byref(self._h), KINDS[kind], 1 if int8 else 0, decimation, taps.data_ptr(), taps.numel(),
                rf_sample_rate, tuning_frequency, ctypes.cast(chans, ctypes.c_void_p), ctypes.cast(dv, ctypes.c_void_p),
                C, first_sample_index, self.device.index))
        else:
            check("gsdrxStreamCreate", lib.gsdrxStreamCreate(
                ctypes.byref(self._h), KINDS[kind], 1 if int8 else 0, decimation, taps.data_ptr(), taps.numel(),
                rf_sample_rate, tuning_frequency, channel_frequency, frequency_deviation, first_sample_index,
                self.device.index))

    def outputs_for(self, num_samples: int) -> int:
        return lib.gsdrxStreamOutputsFor(self._h, num_samples)

    def process(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        want = torch.int8 if self.int8 else torch.complex64
        if x.dtype != want or not x.is_contiguous() or x.device != self.device:
            raise TypeError(f"input must be a contiguous {want} tensor on {self.device}")
        n_in = x.numel() // 2 if self.int8 else x.numel()
        n_out = self.outputs_for(n_in)
        odt = torch.complex64 if self.kind == "fir" else torch.float32
        if self.channels is not None:  # (channels, capacity) rows; the library writes row c at c * capacity
            if out is None:
                out = torch.empty((self.channels, n_out), dtype=odt, device=self.device)
            if out.dtype != odt or out.dim() != 2 or out.shape[0] != self.channels or out.shape[1] < n_out \
                    or not out.is_contiguous():
                raise ValueError(f"output must be a contiguous ({self.channels}, >= {n_out}) {odt} tensor")
            cap = out.shape[1]
        else:
            if out is None:
                out = torch.empty(n_out, dtype=odt, device=self.device)
            if out.dtype != odt or out.numel() < n_out:
                raise ValueError(f"output must hold {n_out} {odt} values")
            cap = out.numel()
        written = ctypes.c_size_t(0)
        check("gsdrxStreamProcess", lib.gsdrxStreamProcess(self._h, x.data_ptr() if n_in else None, n_in,
                                                           out.data_ptr() if n_out else None, cap,
                                                           ctypes.byref(written), stream_of(x)))
        if written.value != n_out:
            raise GsdrError("gsdrxStreamProcess", -1)
        return out[..., :n_out]

    def close(self):
        if self._h:
            check("gsdrxStreamDestroy", lib.gsdrxStreamDestroy(self._h))
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def plan(decimation: int, window: int, consumed: int, next_output: int, chunk: int):
    """gsdrxStreamPlan: (seam outputs, chunk head copied, direct outputs, direct offset, history after)."""
    out = (ctypes.c_uint64 * 5)()
    lib.gsdrxStreamPlan(decimation, window, consumed, next_output, chunk, out)
    return tuple(int(v) for v in out)
