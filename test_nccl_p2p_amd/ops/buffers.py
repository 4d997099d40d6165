"""Payload fill / verification on device tensors.

Device side: the hand-written gfx950 kernels in ``csrc/kernels.hip`` (fill:
16 B/lane stores; verify: register- or LDS-DMA-staged loads with a fused
wave64-shuffle -> LDS -> one-atomic-per-block reduction).  Host side: a plain
PyTorch implementation of the same counter-based PRNG (``csrc/prng.hpp``) so
the kernels can be checked word for word.

The reference benchmark zero-fills its buffers and never reads them back
(/root/reference/p2p_matrix.cc:129-130); this is what replaces that.
"""

from __future__ import annotations

from typing import NamedTuple, Optional

import torch

from .._native import require_native

M32 = 0xFFFFFFFF


def impl_number(name: str) -> int:
    """Verify kernel name -> the native impl number: auto, lds8 (alias lds),
    stride (alias reg); a variant round 5 removed raises ValueError saying so
    (csrc/app.cpp parse_verify_impl, shared with p2p_matrix --verify-impl)."""
    return require_native().parse_verify_impl(name)


class VerifyResult(NamedTuple):
    mismatches: int   # mismatching 32-bit words (tail: partial word counts once)
    checksum: int     # sum of received 32-bit words mod 2**64
    first_bad: int    # lowest mismatching byte offset, 2**64-1 if none

    @property
    def ok(self) -> bool:
        return self.mismatches == 0


def _check_tensor(t: torch.Tensor) -> int:
    if not t.is_cuda:
        raise ValueError("device kernels need a GPU tensor")
    if not t.is_contiguous():
        raise ValueError("tensor must be contiguous")
    if t.data_ptr() % 16:
        raise ValueError("tensor data must be 16-byte aligned (gfx950 dwordx4 accesses)")
    return t.numel() * t.element_size()


def _stream(stream: Optional[torch.cuda.Stream]) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def fill_(t: torch.Tensor, seed: int, stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
    """Fills the bytes of ``t`` with PRNG stream ``seed`` (stream-ordered)."""
    nbytes = _check_tensor(t)
    require_native().fill(t.data_ptr(), nbytes, seed & (2**64 - 1), _stream(stream))
    return t


def verify(t: torch.Tensor, seed: int, impl: str = "auto", stream: Optional[torch.cuda.Stream] = None) -> VerifyResult:
    """Compares ``t`` with PRNG stream ``seed`` on the device (blocking)."""
    nbytes = _check_tensor(t)
    r = require_native().verify(t.data_ptr(), nbytes, seed & (2**64 - 1), impl_number(impl), True, _stream(stream))
    return VerifyResult(*r)


def checksum(t: torch.Tensor, impl: str = "auto", stream: Optional[torch.cuda.Stream] = None) -> int:
    """Sum of the tensor's 32-bit words mod 2**64 (no PRNG compare)."""
    nbytes = _check_tensor(t)
    return int(require_native().verify(t.data_ptr(), nbytes, 0, impl_number(impl), False, _stream(stream))[1])


# ---------------------------------------------------------------- reference --

def _fmix32(h: torch.Tensor) -> torch.Tensor:
    # int64 arithmetic; products wrap mod 2**64 and are masked back to 32 bits.
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & M32
    return h ^ (h >> 16)


def _fmix32_int(h: int) -> int:
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    return h ^ (h >> 16)


def reference_words(start: int, count: int, seed: int, device="cpu") -> torch.Tensor:
    """Words [start, start+count) of the stream as int64 values in [0, 2**32)."""
    seed &= 2**64 - 1
    idx = torch.arange(start, start + count, dtype=torch.int64, device=device)
    hi = idx >> 32
    lo = idx & M32
    seed_lo = seed & M32
    seed_hi = seed >> 32
    inner = _fmix32((seed_hi + hi * 0x27D4EB2F + 0x165667B1) & M32)
    key = _fmix32(seed_lo ^ inner)
    return _fmix32(((lo * 0x9E3779B1) & M32) ^ key)


def reference_bytes(nbytes: int, seed: int, device="cpu") -> torch.Tensor:
    """The first ``nbytes`` of the stream as a uint8 tensor (little-endian words)."""
    nwords = (nbytes + 3) // 4
    w = reference_words(0, nwords, seed, device)
    b = torch.stack([(w >> (8 * k)) & 0xFF for k in range(4)], dim=1).to(torch.uint8).reshape(-1)
    return b[:nbytes]


def reference_verify(data: torch.Tensor, seed: int) -> VerifyResult:
    """PyTorch implementation of the verify kernel's contract on a uint8 tensor."""
    data = data.reshape(-1).to(torch.uint8)
    nbytes = data.numel()
    nwords = (nbytes + 3) // 4
    pad = nwords * 4 - nbytes
    d = torch.cat([data, torch.zeros(pad, dtype=torch.uint8, device=data.device)]).to(torch.int64).reshape(nwords, 4)
    got = d[:, 0] | (d[:, 1] << 8) | (d[:, 2] << 16) | (d[:, 3] << 24)
    want = reference_words(0, nwords, seed, data.device)
    if pad:
        mask = (1 << (8 * (4 - pad))) - 1
        want = want.clone()
        want[-1] &= mask
        got_cmp = got.clone()
        got_cmp[-1] &= mask
    else:
        got_cmp = got
    bad = (got_cmp != want).nonzero().reshape(-1)
    csum = int(got.sum().item()) % 2**64
    first = int(bad[0].item()) * 4 if bad.numel() else 2**64 - 1
    return VerifyResult(int(bad.numel()), csum, first)


def payload_seed(src: int, nbytes: int, salt: int = 0) -> int:
    """Seed of the payload rank ``src`` sends (csrc/prng.hpp payload_seed)."""
    s = 0x9E3779B97F4A7C15 ^ ((src & M32) << 40) ^ nbytes ^ ((salt * 0xD6E8FEB86659FD93) & (2**64 - 1))
    s &= 2**64 - 1
    return s ^ (s >> 29)
