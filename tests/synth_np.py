"""Host (numpy) restatement of the device workload generator
(tcp-stack_amd/csrc/tcpck_synth.hip) -- test infrastructure.

Lets CPU tests build the exact bytes the GPU benchmark checksums, and lets the
GPU tests check the generator itself.  Layout helpers for the BASELINE configs
live here too (fixed stride, and the C3 mixed 64/576/1460-payload batch).
"""
from __future__ import annotations

import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = (x + np.uint64(0x9E3779B97F4A7C15)) & M64
        x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M64
        x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M64
        return x ^ (x >> np.uint64(31))


def header(payload: int, seq: int) -> np.ndarray:
    """The 32-byte network-order header the generator writes (checksum 0)."""
    h = np.zeros(32, np.uint8)
    h[0:4] = [127, 0, 0, 1]
    h[4:8] = [127, 0, 0, 1]
    h[9] = 6
    h[10:12] = [(payload >> 8) & 0xFF, payload & 0xFF]
    h[12:14] = [15500 >> 8, 15500 & 0xFF]
    h[14:16] = [15501 >> 8, 15501 & 0xFF]
    h[16:20] = [(seq >> 24) & 0xFF, (seq >> 16) & 0xFF, (seq >> 8) & 0xFF, seq & 0xFF]
    h[20:24] = [0, 0, 0, 77]
    h[25] = 0x08  # ACK (tcp-header.h:129-134 -> bit 107 of the TCP field)
    h[26:28] = [1024 >> 8, 1024 & 0xFF]
    return h


def image(seed: int, index: int, length: int, kind: int = 0) -> np.ndarray:
    """Bytes of synthetic image `index` of `length` bytes."""
    assert length % 2 == 0
    out = np.zeros(length, np.uint8)
    payload = length - 32 if length >= 32 else 0
    h = header(payload, (1000 + index) & 0xFFFFFFFF)
    n = min(32, length)
    out[:n] = h[:n]
    if length > 32:
        nw = (length - 32) // 2
        if kind == 1:
            pass
        elif kind == 2:
            out[32:] = 0xFF
        else:
            with np.errstate(over="ignore"):
                key = splitmix64(np.array([np.uint64(seed) ^ ((np.uint64(index) * np.uint64(0xD1B54A32D192ED03)) & M64)],
                                          dtype=np.uint64))[0]
            m = np.arange(nw, dtype=np.uint64)
            with np.errstate(over="ignore"):
                r = splitmix64((key + (m >> np.uint64(2))) & M64)
            words = ((r >> (np.uint64(16) * (m & np.uint64(3)))) & np.uint64(0xFFFF)).astype("<u2")
            out[32:32 + 2 * nw] = words.view(np.uint8)
    return out


def arena_fixed(seed: int, count: int, stride: int, length: int, first_index: int = 0,
                kind: int = 0) -> np.ndarray:
    a = np.zeros(count * stride if count else 0, np.uint8)
    for k in range(count):
        a[k * stride:k * stride + length] = image(seed, first_index + k, length, kind)
    return a


C3_PAYLOADS = (64, 576, 1460)


def mixed_layout(count: int, seed: int = 42, payloads=C3_PAYLOADS, align: int = 2):
    """C3: payload i.i.d. uniform over {64, 576, 1460}; packed back to back.

    Returns (offsets u64, lengths u32, total_bytes)."""
    rng = np.random.default_rng(seed)
    lengths = (np.asarray(payloads, np.uint32)[rng.integers(0, len(payloads), count)] + 32).astype(np.uint32)
    padded = ((lengths.astype(np.uint64) + np.uint64(align - 1)) // np.uint64(align)) * np.uint64(align)
    offsets = np.zeros(count, np.uint64)
    if count > 1:
        np.cumsum(padded[:-1], out=offsets[1:])
    total = int(offsets[-1] + padded[-1]) if count else 0
    return offsets, lengths, total
