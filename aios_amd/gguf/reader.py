"""GGUF v2/v3 reader and writer.

The reference never parses GGUF itself: it hands the file path to llama-server
(`runtime/src/model_manager.rs:187-204`).  Our runtime owns the format: the
reader memory-maps the file (no copy of the tensor data section), exposes the
metadata KV table and tensor infos, and hands raw block bytes to the device
loader (`aios_amd.runtime.loader`) which uploads and repacks them in HBM.

The writer is used to emit random-init synthetic models of a named
architecture (TinyLlama / Mistral / Llama-3 / Qwen shapes) for tests and
benchmarks (SURVEY.md §7.3 step 2, §7.5 "Synthetic models").
"""
from __future__ import annotations

import dataclasses
import io
import mmap
import os
import struct
from typing import Any, BinaryIO, Dict, List, Optional

import numpy as np

from .quants import BLOCK_INFO, GGMLType, type_size

GGUF_MAGIC = 0x46554747  # "GGUF" little-endian
DEFAULT_ALIGNMENT = 32


class GGUFValueType:
    UINT8 = 0
    INT8 = 1
    UINT16 = 2
    INT16 = 3
    UINT32 = 4
    INT32 = 5
    FLOAT32 = 6
    BOOL = 7
    STRING = 8
    ARRAY = 9
    UINT64 = 10
    INT64 = 11
    FLOAT64 = 12


_SCALAR_FMT = {
    GGUFValueType.UINT8: "<B", GGUFValueType.INT8: "<b", GGUFValueType.UINT16: "<H",
    GGUFValueType.INT16: "<h", GGUFValueType.UINT32: "<I", GGUFValueType.INT32: "<i",
    GGUFValueType.FLOAT32: "<f", GGUFValueType.BOOL: "<?", GGUFValueType.UINT64: "<Q",
    GGUFValueType.INT64: "<q", GGUFValueType.FLOAT64: "<d",
}
_NP_DTYPE = {
    GGUFValueType.UINT8: np.uint8, GGUFValueType.INT8: np.int8, GGUFValueType.UINT16: np.uint16,
    GGUFValueType.INT16: np.int16, GGUFValueType.UINT32: np.uint32, GGUFValueType.INT32: np.int32,
    GGUFValueType.FLOAT32: np.float32, GGUFValueType.UINT64: np.uint64, GGUFValueType.INT64: np.int64,
    GGUFValueType.FLOAT64: np.float64, GGUFValueType.BOOL: np.bool_,
}


@dataclasses.dataclass
class TensorInfo:
    name: str
    shape: tuple          # ggml order: ne0 (innermost / contiguous) first
    ggml_type: GGMLType
    offset: int           # relative to data section
    nbytes: int

    @property
    def n_elements(self) -> int:
        n = 1
        for s in self.shape:
            n *= s
        return n

    @property
    def rows(self) -> int:
        return self.n_elements // self.shape[0]

    @property
    def cols(self) -> int:
        return self.shape[0]


class GGUFReader:
    """Zero-copy GGUF reader over an mmap."""

    def __init__(self, path: str):
        self.path = path
        self._f = open(path, "rb")
        self._mm = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_READ)
        self.metadata: Dict[str, Any] = {}
        self.metadata_types: Dict[str, int] = {}
        self.tensors: Dict[str, TensorInfo] = {}
        self._parse()

    # -- low level -------------------------------------------------------------------
    def _read(self, fmt: str):
        v = struct.unpack_from(fmt, self._mm, self._pos)
        self._pos += struct.calcsize(fmt)
        return v[0]

    def _read_str(self) -> str:
        n = self._read("<Q")
        s = bytes(self._mm[self._pos:self._pos + n])
        self._pos += n
        return s.decode("utf-8", errors="replace")

    def _read_value(self, vtype: int):
        if vtype == GGUFValueType.STRING:
            return self._read_str()
        if vtype == GGUFValueType.ARRAY:
            etype = self._read("<I")
            n = self._read("<Q")
            if etype == GGUFValueType.STRING:
                return [self._read_str() for _ in range(n)]
            if etype == GGUFValueType.ARRAY:
                return [self._read_value(GGUFValueType.ARRAY) for _ in range(n)]
            dt = np.dtype(_NP_DTYPE[etype])
            arr = np.frombuffer(self._mm, dtype=dt, count=n, offset=self._pos).copy()
            self._pos += n * dt.itemsize
            return arr
        return self._read(_SCALAR_FMT[vtype])

    def _parse(self):
        self._pos = 0
        magic = self._read("<I")
        if magic != GGUF_MAGIC:
            raise ValueError(f"{self.path}: not a GGUF file (magic {magic:#x})")
        self.version = self._read("<I")
        if self.version not in (2, 3):
            raise ValueError(f"unsupported GGUF version {self.version}")
        n_tensors = self._read("<Q")
        n_kv = self._read("<Q")
        for _ in range(n_kv):
            key = self._read_str()
            vtype = self._read("<I")
            self.metadata[key] = self._read_value(vtype)
            self.metadata_types[key] = vtype
        infos = []
        for _ in range(n_tensors):
            name = self._read_str()
            nd = self._read("<I")
            shape = tuple(self._read("<Q") for _ in range(nd))
            t = GGMLType(self._read("<I"))
            off = self._read("<Q")
            infos.append((name, shape, t, off))
        self.alignment = int(self.metadata.get("general.alignment", DEFAULT_ALIGNMENT))
        self.data_offset = (self._pos + self.alignment - 1) // self.alignment * self.alignment
        for name, shape, t, off in infos:
            n = int(np.prod(shape))
            self.tensors[name] = TensorInfo(name, shape, t, off, type_size(t, n))

    # -- public ----------------------------------------------------------------------
    @property
    def architecture(self) -> str:
        return str(self.metadata.get("general.architecture", "llama"))

    def get(self, key: str, default=None):
        return self.metadata.get(key, default)

    def arch_get(self, key: str, default=None):
        return self.metadata.get(f"{self.architecture}.{key}", default)

    def tensor_bytes(self, name: str) -> memoryview:
        ti = self.tensors[name]
        start = self.data_offset + ti.offset
        return memoryview(self._mm)[start:start + ti.nbytes]

    def tensor_array(self, name: str) -> np.ndarray:
        """Raw uint8 view (zero-copy) of a tensor's blocks."""
        return np.frombuffer(self.tensor_bytes(name), dtype=np.uint8)

    def dequantize(self, name: str) -> np.ndarray:
        from .quants import dequantize
        ti = self.tensors[name]
        return dequantize(self.tensor_array(name), ti.ggml_type, tuple(reversed(ti.shape)))

    def close(self):
        try:
            self._mm.close()
        except BufferError:
            pass  # outstanding numpy views keep the map alive; the GC closes it
        self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class GGUFWriter:
    """Streaming GGUF v3 writer.  Tensors are given as raw block bytes + ggml shape."""

    def __init__(self, path: str, alignment: int = DEFAULT_ALIGNMENT):
        self.path = path
        self.alignment = alignment
        self.kv: List[tuple] = []
        self.tensors: List[tuple] = []  # (name, shape, type, raw bytes or callable)

    def add(self, key: str, value: Any, vtype: Optional[int] = None):
        if vtype is None:
            vtype = self._infer_type(value)
        self.kv.append((key, vtype, value))

    @staticmethod
    def _infer_type(value) -> int:
        if isinstance(value, bool):
            return GGUFValueType.BOOL
        if isinstance(value, int):
            return GGUFValueType.UINT32 if 0 <= value < 2 ** 32 else GGUFValueType.INT64
        if isinstance(value, float):
            return GGUFValueType.FLOAT32
        if isinstance(value, str):
            return GGUFValueType.STRING
        if isinstance(value, (list, tuple, np.ndarray)):
            return GGUFValueType.ARRAY
        raise TypeError(type(value))

    def add_tensor(self, name: str, shape: tuple, ggml_type: GGMLType, raw: np.ndarray):
        """shape in ggml order (ne0 first)."""
        n = int(np.prod(shape))
        expect = type_size(ggml_type, n)
        raw = np.ascontiguousarray(raw).view(np.uint8).ravel()
        if raw.size != expect:
            raise ValueError(f"{name}: {raw.size} bytes, expected {expect}")
        self.tensors.append((name, tuple(int(s) for s in shape), GGMLType(ggml_type), raw))

    # -- serialisation ---------------------------------------------------------------
    @staticmethod
    def _w_str(f: BinaryIO, s: str):
        b = s.encode("utf-8")
        f.write(struct.pack("<Q", len(b)))
        f.write(b)

    def _w_value(self, f: BinaryIO, vtype: int, value):
        if vtype == GGUFValueType.STRING:
            self._w_str(f, value)
        elif vtype == GGUFValueType.ARRAY:
            items = list(value) if not isinstance(value, np.ndarray) else value
            if isinstance(items, np.ndarray):
                etype = {np.dtype(v): k for k, v in _NP_DTYPE.items()}.get(items.dtype)
                if etype is None:
                    raise TypeError(items.dtype)
                f.write(struct.pack("<IQ", etype, items.size))
                f.write(np.ascontiguousarray(items).tobytes())
                return
            if len(items) and isinstance(items[0], str):
                f.write(struct.pack("<IQ", GGUFValueType.STRING, len(items)))
                for s in items:
                    self._w_str(f, s)
                return
            etype = GGUFValueType.INT32 if all(isinstance(i, int) for i in items) else GGUFValueType.FLOAT32
            f.write(struct.pack("<IQ", etype, len(items)))
            for i in items:
                f.write(struct.pack(_SCALAR_FMT[etype], i))
        else:
            f.write(struct.pack(_SCALAR_FMT[vtype], value))

    def write(self):
        with open(self.path, "wb") as f:
            f.write(struct.pack("<IIQQ", GGUF_MAGIC, 3, len(self.tensors), len(self.kv) + 1))
            self._w_str(f, "general.alignment")
            f.write(struct.pack("<I", GGUFValueType.UINT32))
            f.write(struct.pack("<I", self.alignment))
            for key, vtype, value in self.kv:
                self._w_str(f, key)
                f.write(struct.pack("<I", vtype))
                self._w_value(f, vtype, value)
            offset = 0
            offsets = []
            for name, shape, t, raw in self.tensors:
                offsets.append(offset)
                offset += (raw.size + self.alignment - 1) // self.alignment * self.alignment
            for (name, shape, t, raw), off in zip(self.tensors, offsets):
                self._w_str(f, name)
                f.write(struct.pack("<I", len(shape)))
                for s in shape:
                    f.write(struct.pack("<Q", s))
                f.write(struct.pack("<IQ", int(t), off))
            pos = f.tell()
            pad = (pos + self.alignment - 1) // self.alignment * self.alignment - pos
            f.write(b"\0" * pad)
            for (name, shape, t, raw), off in zip(self.tensors, offsets):
                f.write(raw.tobytes())
                pad = (raw.size + self.alignment - 1) // self.alignment * self.alignment - raw.size
                f.write(b"\0" * pad)
