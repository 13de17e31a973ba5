"""tcpck -- Python binding of libtcpck.so (the MI355X TCP checksum library).

A thin ctypes layer over the C ABI declared in include/tcpck.h, used by the
parity tests and bench.py.  There is no Python or CPU fallback for the batched
path: if libtcpck.so is missing or the device is not a gfx950, constructing a
``Context`` raises.

libtcpck.so holds the kernels the AUTO policy can pick; its tcpck_tuning.h
entry points (``batch_*_ex``) accept only those.  ``Context(probe=True)``
binds libtcpck_probe.so instead: the same sources built with every measured
variant, the per-wave time stamps and the diag kernels (scripts/, the
variant tests).

Reference API mirrored (filixi/TCP-stack):
  * ``checksum16``   <- CalculateChecksum(const TcpPacket&), include/tcp-header.h:252-263
  * OP_FILL          <- Checksum()=0; Checksum()=CalculateChecksum(pkt),
                        src/socket-manager.cc:9-10, include/socket-manager.h:259-260
  * OP_VERIFY        <- CalculateChecksum(pkt) == 0, include/socket-manager.h:182
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
LIB_PATH = os.path.join(PKG_ROOT, "libtcpck.so")
# tests/test_abi_asan.py only: the same product library with its host code
# built under ASan + UBSan (tcp-stack_amd/Makefile `asan`), loaded in place of
# libtcpck.so by a python started with the sanitizer runtime preloaded
ASAN_PATH = os.path.join(PKG_ROOT, "libtcpck_asan.so")
if os.environ.get("TCPCK_LIB_VARIANT") == "asan":
    LIB_PATH = ASAN_PATH
PROBE_PATH = os.path.join(PKG_ROOT, "libtcpck_probe.so")

OK = 0
EINVAL = -22
ENOMEM = -12
ENODEV = -19
EHIP = -1000

MODE_REF = 0
MODE_RFC1071 = 1

OP_CHECKSUM = 0
OP_FILL = 1
OP_VERIFY = 2
OP_RECEIVE = 3  # VERIFY + TcpHeaderN2H in place (device batches)
HEADER_BYTES = 32

LAYOUT_PACKED = 1
LAYOUT_SORTED = 2

# include/tcpck_tuning.h
KERNEL_AUTO = 0
KERNEL_SEG = 1    # param: seg shape + 1 (1..11, SEG_SHAPES), 0 = by length
KERNEL_RSTREAM = 5  # fixed stride == len: param = variant (10 = policy) | cap << 8 | oversub << 16
KERNEL_VVSTREAM = 8  # packed variable or fixed (stride >= len): param = 0/1 U4/U8 byte split, 2/3 count split, 4 policy | oversub << 16
KERNEL_GSTREAM = 9  # fixed stride == len, len a power of two in [32, 1024], 16-B aligned arena: param = 0/1/2 U4/U8/U2 (+4 default block order) | oversub << 16
KERNEL_PATCH = 12  # libtcpck_probe.so only (tcpck_probe.h): FILL's deferred field pass alone
KERNEL_SSTREAM = 10  # slotted layouts (fixed slots, stride % 16 == 0, or any offset list): param = 0 policy (U4, scattered order), 1 U4, 2 U8 (+4 default block order, +8 scattered) | oversub << 16
KERNEL_RVSTREAM = 13  # packed offset lists, REF, CHECKSUM / VERIFY: rstream's scalar walk over the lengths
SEG_SHAPES = {1: "G8/U2", 2: "G16/U6", 3: "G64/U4", 4: "G64/U2", 5: "G32/U3", 6: "G4/U8", 7: "W4/U4", 8: "W8/U4", 9: "W16/U2", 10: "W16/U4", 11: "W2/U4"}
# include/tcpck_tuning.h: in libtcpck.so (AUTO's kernels only) and libtcpck_probe.so
TUNING_EXPORTS = ("tcpck_batch_fixed_ex", "tcpck_batch_var_ex", "tcpck_batch_segment_ex", "tcpck_batch_receive_ex")
# include/tcpck_tuning.h, measurement only: libtcpck_probe.so
PROBE_EXPORTS = ("tcpck_ctx_set_debug", "tcpck_diag_stream", "tcpck_probe_receive_ex", "tcpck_probe_scratch_state",
                 "tcpck_probe_scratch_fail", "tcpck_probe_set_fill_pipe")
# include/tcpck_probe.h: tcpck_probe_receive_ex's flags word (the header pass forms)
PROBE_RECEIVE_HDR_FIRST = 1    # accepted, no effect (the product's separate header pass runs first since round 5)
PROBE_PARAM_PATCH_REVERSE = 1 << 27  # tcpck_batch_*_ex param (probe library): FILL's field pass in reverse order
PROBE_PIPE_ONE_STREAM = 0x100  # set_fill_pipe(k | this): the k chunks on the caller's stream only
PROBE_RECEIVE_HDR_AFTER = 16   # the separate header pass after VERIFY (the order before round 5)
PROBE_RECEIVE_CONCURRENT = 2   # header pass on a side stream beside VERIFY
PROBE_RECEIVE_HDR_WT = 4       # header array stores written through
PROBE_RECEIVE_HDR_WIDE = 8     # two lanes per image, 16-B loads with cache bits (flags >> 4) & 3
PROBE_RECEIVE_ORDER_SHIFT = 8  # (flags >> 8) & 3: header pass image order (1 XCD-chunked, 2 scattered, 3 transposed)
# Kernel params libtcpck.so runs (the AUTO policy's own choices, tcpck_api.hip
# run_fixed_impl / run_var_impl); every other value needs libtcpck_probe.so.
SEG_AUTO_SHAPES = (0, 1, 2, 7, 8, 9, 11)  # by length, G8/U2, G16/U6, W4, W8, W16, W2 (shape_for_len)
RSTREAM_AUTO = (20, 25)                   # the policy; 25: its FILL with the write-through 2-B field pass
GSTREAM_AUTO = (0, 0x80, 0x401)           # (+ 4: default block order)
SSTREAM_AUTO = (0, 32, 128)               # the policy; + 32: RECEIVE headers from the stream; + 128: FILL's deferred fields


def in_product(kernel: int, param: int, op: int | None = None) -> bool:
    """Whether libtcpck.so runs `kernel` with `param` (tcpck_tuning.h) for `op`."""
    if kernel == KERNEL_AUTO:
        return True
    if kernel == KERNEL_PATCH:
        return False
    if kernel == KERNEL_SEG:
        return (param & 0xFF) in SEG_AUTO_SHAPES
    if kernel == KERNEL_RSTREAM:
        return (param & 0xFF) in RSTREAM_AUTO
    if kernel == KERNEL_VVSTREAM:
        return (param & 7) == 4
    if kernel == KERNEL_GSTREAM:  # AUTO's FILL only
        return (param & 0xFFFF & ~4) in GSTREAM_AUTO and op in (None, OP_FILL)
    if kernel == KERNEL_SSTREAM:
        return (param & 0xFF) in SSTREAM_AUTO
    return True  # unknown kernels: both libraries reject them


def segment_in_product(param: int) -> bool:
    """Whether libtcpck.so runs tcpck_batch_segment_ex with `param` (0: the policy; + 8: default order)."""
    return (param & 7) == 0


PARAM_FILL_UPDATE = 1 << 28  # FILL: the kernel's CHECKSUM pass + the field-update pass
PARAM_FILL_INSTREAM = 1 << 29  # FILL under AUTO: the field zeroed in the stream
PARAM_RECEIVE_TWO_PASS = 1 << 30  # RECEIVE into a header array: separate header pass

# Every symbol include/tcpck.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "tcpck_abi_version", "tcpck_strerror", "tcpck_device_supported",
    "tcpck_ctx_create", "tcpck_ctx_destroy", "tcpck_ctx_device",
    "tcpck_checksum16", "tcpck_fill16", "tcpck_update16",
    "tcpck_batch_fixed", "tcpck_batch_var", "tcpck_batch_set_ack",
    "tcpck_host_batch_fixed", "tcpck_host_batch_var", "tcpck_ctx_set_chunk_bytes",
    "tcpck_host_alloc", "tcpck_host_free", "tcpck_device_alloc", "tcpck_device_free",
    "tcpck_memcpy_h2d", "tcpck_memcpy_d2h", "tcpck_stream_sync",
    "tcpck_synth_fixed", "tcpck_synth_var", "tcpck_batch_segment", "tcpck_batch_header_swap",
    "tcpck_batch_receive", "tcpck_host_batch_fixed_multi", "tcpck_host_batch_var_multi",
)


class TcpckError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{what}: status {status} ({strerror(status)})")


class Layout(ctypes.Structure):
    _fields_ = [("total_bytes", ctypes.c_uint64), ("min_len", ctypes.c_uint32),
                ("max_len", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


_libs: dict = {}


def lib(probe: bool = False) -> ctypes.CDLL:
    """Loads libtcpck.so (probe: libtcpck_probe.so), built in-tree by
    __graft_entry__.build(); raises if absent."""
    if probe in _libs:
        return _libs[probe]
    path = PROBE_PATH if probe else LIB_PATH
    if not os.path.exists(path):
        raise ImportError(f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(path)
    vp, u64, u32, i32, sz = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_size_t
    sig = {
        "tcpck_abi_version": (i32, []),
        "tcpck_strerror": (ctypes.c_char_p, [i32]),
        "tcpck_device_supported": (i32, [i32]),
        "tcpck_ctx_create": (i32, [i32, ctypes.POINTER(vp)]),
        "tcpck_ctx_destroy": (i32, [vp]),
        "tcpck_ctx_device": (i32, [vp]),
        "tcpck_checksum16": (i32, [vp, sz, i32, ctypes.POINTER(ctypes.c_uint16)]),
        "tcpck_fill16": (i32, [vp, sz, i32, ctypes.POINTER(ctypes.c_uint16)]),
        "tcpck_update16": (ctypes.c_uint16, [ctypes.c_uint16, ctypes.c_uint16, ctypes.c_uint16, i32]),
        "tcpck_batch_fixed": (i32, [vp, i32, i32, vp, u64, u32, u64, vp, vp]),
        "tcpck_batch_var": (i32, [vp, i32, i32, vp, vp, vp, u64, vp, ctypes.POINTER(Layout), vp]),
        "tcpck_batch_set_ack": (i32, [vp, i32, vp, vp, u64, u64, vp, u32, vp, vp]),
        "tcpck_host_batch_fixed": (i32, [vp, i32, i32, vp, u64, u32, u64, vp]),
        "tcpck_host_batch_var": (i32, [vp, i32, i32, vp, vp, vp, u64, vp]),
        "tcpck_host_batch_fixed_multi": (i32, [ctypes.POINTER(vp), i32, i32, i32, vp, u64, u32, u64, vp]),
        "tcpck_host_batch_var_multi": (i32, [ctypes.POINTER(vp), i32, i32, i32, vp, vp, vp, u64, vp]),
        "tcpck_ctx_set_chunk_bytes": (i32, [vp, u64]),
        "tcpck_host_alloc": (i32, [sz, ctypes.POINTER(vp)]),
        "tcpck_host_free": (i32, [vp]),
        "tcpck_device_alloc": (i32, [vp, sz, ctypes.POINTER(vp)]),
        "tcpck_device_free": (i32, [vp, vp]),
        "tcpck_memcpy_h2d": (i32, [vp, vp, vp, sz]),
        "tcpck_memcpy_d2h": (i32, [vp, vp, vp, sz]),
        "tcpck_stream_sync": (i32, [vp, vp]),
        "tcpck_synth_fixed": (i32, [vp, u64, u32, u64, u64, u64, i32, vp]),
        "tcpck_synth_var": (i32, [vp, vp, vp, u32, u64, u64, u64, i32, vp]),
        "tcpck_batch_segment": (i32, [vp, i32, vp, u64, u32, vp, u32, vp, u64, vp, vp]),
        "tcpck_batch_segment_ex": (i32, [vp, i32, vp, u64, u32, vp, u32, vp, u64, vp, i32, vp]),
        "tcpck_batch_header_swap": (i32, [vp, vp, vp, u64, u64, vp]),
        "tcpck_batch_receive": (i32, [vp, i32, vp, u64, u32, vp, vp, u64, vp, vp, ctypes.POINTER(Layout), vp]),
        "tcpck_batch_receive_ex": (i32, [vp, i32, vp, u64, u32, vp, vp, u64, vp, vp, ctypes.POINTER(Layout), i32, i32,
                                         vp]),
        # include/tcpck_tuning.h
        "tcpck_batch_fixed_ex": (i32, [vp, i32, i32, vp, u64, u32, u64, vp, i32, i32, vp]),
        "tcpck_batch_var_ex": (i32, [vp, i32, i32, vp, vp, vp, u64, vp, ctypes.POINTER(Layout), i32, i32, vp]),
        "tcpck_ctx_set_debug": (i32, [vp, vp]),
        "tcpck_probe_scratch_state": (i32, [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]),
        "tcpck_probe_scratch_fail": (i32, [vp, i32, ctypes.POINTER(u64)]),
        "tcpck_probe_set_fill_pipe": (i32, [vp, i32, i32]),
        "tcpck_diag_stream": (i32, [vp, i32, vp, u64, vp, vp]),
        "tcpck_probe_receive_ex": (i32, [vp, i32, vp, u64, u32, vp, vp, u64, vp, vp, ctypes.POINTER(Layout), i32, i32,
                                         i32, vp]),
    }
    for name, (res, args) in sig.items():
        if name in PROBE_EXPORTS and not probe:
            continue  # measurement-only: not in the product library
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _libs[probe] = L
    return L


def probe_lib() -> ctypes.CDLL:
    """libtcpck_probe.so (every measured kernel variant; tcpck_tuning.h in full)."""
    return lib(probe=True)


def strerror(status: int) -> str:
    try:
        return lib().tcpck_strerror(status).decode()
    except ImportError:
        return "libtcpck.so unavailable"


def _check(status: int, what: str) -> None:
    if status != OK:
        raise TcpckError(status, what)


def _ptr(x) -> int | None:
    """Device/host address of a torch tensor, numpy array or int (None -> NULL)."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    raise TypeError(f"cannot take the address of {type(x)}")


def _stream(s) -> int | None:
    if s is None:
        return None
    if isinstance(s, int):
        return s
    return s.cuda_stream  # torch.cuda.Stream


# ---- single image, host ------------------------------------------------------

def _as_u8(buf):
    import numpy as np
    if isinstance(buf, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(buf), dtype=np.uint8)
    return np.ascontiguousarray(buf, dtype=np.uint8)


def checksum16(buf, mode: int = MODE_REF) -> int:
    """CalculateChecksum of one host image (tcp-header.h:252-263)."""
    a = _as_u8(buf)
    out = ctypes.c_uint16()
    _check(lib().tcpck_checksum16(a.ctypes.data, a.size, mode, ctypes.byref(out)), "tcpck_checksum16")
    return out.value


def fill16(img, mode: int = MODE_REF) -> int:
    """Send-side insertion in place on a writable uint8 numpy image."""
    out = ctypes.c_uint16()
    _check(lib().tcpck_fill16(img.ctypes.data, img.size, mode, ctypes.byref(out)), "tcpck_fill16")
    return out.value


def update16(checksum: int, old_word: int, new_word: int, mode: int = MODE_REF) -> int:
    return int(lib().tcpck_update16(checksum, old_word, new_word, mode))


def synth_fixed(arena, stride: int, length: int, count: int, seed: int = 42,
                first_index: int = 0, kind: int = 0, stream=None) -> None:
    """Fills a device arena with a fixed-stride synthetic batch (see include/tcpck.h)."""
    _check(lib().tcpck_synth_fixed(_ptr(arena), stride, length, count, seed, first_index, kind,
                                   _stream(stream)), "tcpck_synth_fixed")


def synth_var(arena, offsets, lengths, max_len: int, count: int, seed: int = 42,
              first_index: int = 0, kind: int = 0, stream=None) -> None:
    _check(lib().tcpck_synth_var(_ptr(arena), _ptr(offsets), _ptr(lengths), max_len, count, seed,
                                 first_index, kind, _stream(stream)), "tcpck_synth_var")


# ---- context -------------------------------------------------------------------

class Context:
    """One libtcpck context bound to a HIP device (gfx950 only)."""

    def __init__(self, device: int = 0, probe: bool = False):
        self._h = ctypes.c_void_p()
        self._L = lib(probe)
        self.probe = probe
        _check(self._L.tcpck_ctx_create(device, ctypes.byref(self._h)), f"tcpck_ctx_create({device})")
        self.device = device

    def close(self) -> None:
        if self._h:
            self._L.tcpck_ctx_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # device-resident batches (the hot path)
    def batch_fixed(self, op: int, arena, stride: int, length: int, count: int, out,
                    mode: int = MODE_REF, stream=None) -> None:
        _check(self._L.tcpck_batch_fixed(self._h, op, mode, _ptr(arena), stride, length, count,
                                       _ptr(out), _stream(stream)), "tcpck_batch_fixed")

    def batch_var(self, op: int, arena, offsets, lengths, count: int, out, mode: int = MODE_REF,
                  total_bytes: int = 0, min_len: int = 0, max_len: int = 0, packed: bool = False,
                  sorted: bool = False, stream=None) -> None:
        lay = Layout(total_bytes, min_len, max_len,
                     (LAYOUT_PACKED if packed else 0) | (LAYOUT_SORTED if sorted else 0), 0)
        _check(self._L.tcpck_batch_var(self._h, op, mode, _ptr(arena), _ptr(offsets), _ptr(lengths),
                                     count, _ptr(out), ctypes.byref(lay), _stream(stream)),
               "tcpck_batch_var")

    def batch_set_ack(self, arena, count: int, ack: int = 0, acks=None, offsets=None, stride: int = 0,
                      out=None, mode: int = MODE_REF, stream=None) -> None:
        """Retransmit batch (socket-internal.h:376-377 + socket-manager.cc:9-10): bytes 20-23 of every
        image := htonl(ack or acks[k]), checksum at 28-29 updated incrementally (tcpck_batch_set_ack)."""
        _check(self._L.tcpck_batch_set_ack(self._h, mode, _ptr(arena), _ptr(offsets), stride, count,
                                         _ptr(acks), ack & 0xFFFFFFFF, _ptr(out), _stream(stream)),
               "tcpck_batch_set_ack")

    def batch_header_swap(self, arena, count: int, offsets=None, stride: int = 0, stream=None) -> None:
        """TcpHeaderN2H (== TcpHeaderH2N, tcp-header.h:193-221) in place on the first 32 bytes of
        every image (tcpck_batch_header_swap); after VERIFY this completes ReceivePacket's
        front half (socket-manager.h:182-184)."""
        _check(self._L.tcpck_batch_header_swap(self._h, _ptr(arena), _ptr(offsets), stride, count,
                                             _stream(stream)), "tcpck_batch_header_swap")

    def batch_receive(self, arena, count: int, ok, hdr=None, stride: int = 0, length: int = 0, offsets=None,
                      lengths=None, mode: int = MODE_REF, total_bytes: int = 0, min_len: int = 0, max_len: int = 0,
                      packed: bool = False, sorted: bool = False, stream=None, kernel: int | None = None,
                      param: int = 0, probe_flags: int | None = None) -> None:
        """ReceivePacket's front half for a batch (tcpck_batch_receive): ok[k] = verdict on the
        network-order image; headers in host order in place (hdr None) or into hdr (32 B per image,
        the arena left as received).  Fixed layout (stride, length) or offsets + lengths.
        kernel/param: tcpck_batch_receive_ex (include/tcpck_tuning.h); probe_flags (probe contexts
        only): tcpck_probe_receive_ex's header pass forms (PROBE_RECEIVE_*, include/tcpck_probe.h)."""
        lay = Layout(total_bytes, min_len, max_len,
                     (LAYOUT_PACKED if packed else 0) | (LAYOUT_SORTED if sorted else 0), 0)
        args = (self._h, mode, _ptr(arena), stride, length, _ptr(offsets), _ptr(lengths), count, _ptr(ok), _ptr(hdr),
                ctypes.byref(lay))
        if probe_flags is not None:
            _check(self._L.tcpck_probe_receive_ex(*args, kernel or KERNEL_AUTO, param, probe_flags, _stream(stream)),
                   "tcpck_probe_receive_ex")
        elif kernel is None:
            _check(self._L.tcpck_batch_receive(*args, _stream(stream)), "tcpck_batch_receive")
        else:
            _check(self._L.tcpck_batch_receive_ex(*args, kernel, param, _stream(stream)), "tcpck_batch_receive_ex")

    def batch_segment(self, payload, payload_bytes: int, seg: int, hdr, seq0: int, images, stride: int,
                      out=None, mode: int = MODE_REF, param: int | None = None, stream=None) -> int:
        """Send stream -> checksummed images (tcpck_batch_segment): image k at k * stride
        = hdr with TcpLength/seq of segment k + payload[k seg, ...), checksum filled.
        hdr: 32 bytes (network order).  Returns the number of images."""
        h = _as_u8(hdr)
        if h.size != 32:
            raise ValueError("hdr must be 32 bytes")
        args = (self._h, mode, _ptr(payload), payload_bytes, seg, h.ctypes.data, seq0 & 0xFFFFFFFF, _ptr(images),
                stride, _ptr(out))
        if param is None:
            _check(self._L.tcpck_batch_segment(*args, _stream(stream)), "tcpck_batch_segment")
        else:
            _check(self._L.tcpck_batch_segment_ex(*args, param, _stream(stream)), "tcpck_batch_segment_ex")
        return (payload_bytes + seg - 1) // seg

    # explicit kernel choice (include/tcpck_tuning.h)
    def batch_fixed_ex(self, op: int, arena, stride: int, length: int, count: int, out, kernel: int,
                       param: int = 0, mode: int = MODE_REF, stream=None) -> None:
        _check(self._L.tcpck_batch_fixed_ex(self._h, op, mode, _ptr(arena), stride, length, count,
                                          _ptr(out), kernel, param, _stream(stream)), "tcpck_batch_fixed_ex")

    def batch_var_ex(self, op: int, arena, offsets, lengths, count: int, out, kernel: int,
                     param: int = 0, mode: int = MODE_REF, total_bytes: int = 0, min_len: int = 0,
                     max_len: int = 0, packed: bool = False, sorted: bool = False, stream=None) -> None:
        lay = Layout(total_bytes, min_len, max_len,
                     (LAYOUT_PACKED if packed else 0) | (LAYOUT_SORTED if sorted else 0), 0)
        _check(self._L.tcpck_batch_var_ex(self._h, op, mode, _ptr(arena), _ptr(offsets), _ptr(lengths),
                                        count, _ptr(out), ctypes.byref(lay), kernel, param,
                                        _stream(stream)), "tcpck_batch_var_ex")

    # host-memory batches (end to end, PCIe included)
    def host_batch_fixed(self, op: int, arena, stride: int, length: int, count: int, out,
                         mode: int = MODE_REF) -> None:
        _check(self._L.tcpck_host_batch_fixed(self._h, op, mode, _ptr(arena), stride, length, count,
                                            _ptr(out)), "tcpck_host_batch_fixed")

    def host_batch_var(self, op: int, arena, offsets, lengths, count: int, out,
                       mode: int = MODE_REF) -> None:
        _check(self._L.tcpck_host_batch_var(self._h, op, mode, _ptr(arena), _ptr(offsets),
                                          _ptr(lengths), count, _ptr(out)), "tcpck_host_batch_var")

    def diag_stream(self, variant: int, buf, nbytes: int, out, stream=None) -> None:
        """Timing-only streaming micro-kernel (include/tcpck_tuning.h)."""
        _check(self._L.tcpck_diag_stream(self._h, variant, _ptr(buf), nbytes, _ptr(out), _stream(stream)),
               "tcpck_diag_stream")

    def set_debug(self, buf) -> None:
        """Per-wave {start, end, hw_id, xcc_id} stamp buffer for timing builds (None = off)."""
        _check(self._L.tcpck_ctx_set_debug(self._h, _ptr(buf)), "tcpck_ctx_set_debug")

    def scratch_state(self) -> tuple[int, int]:
        """(slots allocated, bit mask of slots used) of the out-less FILL results
        scratch (libtcpck_probe.so only, tcpck_probe.h)."""
        a, m = ctypes.c_int(), ctypes.c_int()
        _check(self._L.tcpck_probe_scratch_state(self._h, ctypes.byref(a), ctypes.byref(m)),
               "tcpck_probe_scratch_state")
        return a.value, m.value

    def scratch_fail(self, n: int) -> int:
        """Refuse the next n scratch allocations (fault injection, libtcpck_probe.so only);
        returns the refusals so far."""
        r = ctypes.c_uint64()
        _check(self._L.tcpck_probe_scratch_fail(self._h, n, ctypes.byref(r)), "tcpck_probe_scratch_fail")
        return r.value

    def set_fill_pipe(self, k: int, prio: int = 0) -> None:
        """The pipelined FILL under AUTO in this context: k chunks (0/1 serial, -1 AUTO's rule), the
        field passes on a context stream of priority prio (libtcpck_probe.so only, tcpck_probe.h)."""
        _check(self._L.tcpck_probe_set_fill_pipe(self._h, k, prio), "tcpck_probe_set_fill_pipe")

    def set_chunk_bytes(self, n: int) -> None:
        _check(self._L.tcpck_ctx_set_chunk_bytes(self._h, n), "tcpck_ctx_set_chunk_bytes")


def _ctx_array(ctxs):
    if len({c.probe for c in ctxs}) > 1:
        raise ValueError("contexts of libtcpck.so and libtcpck_probe.so cannot be mixed")
    arr = (ctypes.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    return ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)), arr


def host_batch_fixed_multi(ctxs, op: int, arena, stride: int, length: int, count: int, out,
                           mode: int = MODE_REF) -> None:
    """tcpck_host_batch_fixed over several contexts (one per GPU): contiguous equal shards, one host thread each."""
    p, keep = _ctx_array(ctxs)
    _check(ctxs[0]._L.tcpck_host_batch_fixed_multi(p, len(ctxs), op, mode, _ptr(arena), stride, length, count, _ptr(out)),
           "tcpck_host_batch_fixed_multi")
    del keep


def host_batch_var_multi(ctxs, op: int, arena, offsets, lengths, count: int, out, mode: int = MODE_REF) -> None:
    """tcpck_host_batch_var over several contexts: contiguous shards balanced by bytes."""
    p, keep = _ctx_array(ctxs)
    _check(ctxs[0]._L.tcpck_host_batch_var_multi(p, len(ctxs), op, mode, _ptr(arena), _ptr(offsets), _ptr(lengths), count,
                                            _ptr(out)), "tcpck_host_batch_var_multi")
    del keep
