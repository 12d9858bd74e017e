"""Device-resident tracker <-> mapper state exchange.

Drop-in for the reference's `ShareData` (src/share.py:27-166), which
voxslam.py:28-33 serves from a multiprocessing BaseManager: there
`update_share_data` (mapping.py:236-248) deep-copies the decoder and every
map_states tensor to the host and pickles them into the manager, and
`do_tracking` (tracking.py:114-125) pickles them back and re-uploads them
with `.cuda()` — a full host round trip of the map per tracked frame.

Here the same properties (`decoder`, `points_encoder`, `states`, `voxels`,
`octree`, `hash_voxel`, `stop_mapping`, `stop_tracking`,
`tracking_trajectory`, `push_pose`) sit on libpsvo's share channels
(csrc/share.cpp): a setter copies the tensors device-to-device into a slot of
the writer's HBM exported over HIP IPC, a getter copies the latest complete
snapshot device-to-device into fresh tensors of the reader (the reference's
deepcopy semantics).  Nothing crosses PCIe; the only host data are a few
hundred bytes of layout per snapshot.

A ShareData pickles as its shared-memory name, so it can be handed to
`torch.multiprocessing` / `multiprocessing` children exactly as the
reference hands its manager proxy to `Mapping.spin` / `Tracking.spin`.
One writer per channel (the mapper); any number of readers.
"""
from __future__ import annotations

import copy
import ctypes
import json
import os
import pickle
import struct
import uuid

import numpy as np
import torch

from . import _lib as L

CHANNELS = {"decoder": 0, "points_encoder": 1, "states": 2, "voxels": 3, "octree": 4, "hash_voxel": 5}
FLAGS = {"stop_mapping": 0, "stop_tracking": 1}
META_CAP = 65536
POSE_DIM = 8  # trajectory rows [n, pose[0..n), 0...] (include/psvo.h)
PUBLISH_TIMEOUT_MS = 10000

_DTYPES = {str(d): d for d in (torch.float32, torch.float64, torch.float16, torch.bfloat16, torch.int64,
                                torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool)}


def _check(rc, what):
    if rc != 0:
        raise L.PsvoError(f"{what} failed (code {rc}): {L.lib().psvo_last_error().decode(errors='replace')}")


_SKELETONS = {}   # last module skeleton published by this process (the mapper republishes one decoder)


def _flatten(value):
    """value -> (kind, [(name, tensor)], skeleton bytes)."""
    if value is None:
        return "none", [], b""
    if isinstance(value, torch.Tensor):
        return "tensor", [("", value)], b""
    if isinstance(value, torch.nn.Module):
        # structure without storage: the reader materialises it with to_empty()
        items = list(value.state_dict().items())
        sig = (id(value), type(value), tuple((k, tuple(t.shape), t.dtype) for k, t in items))
        skel = _SKELETONS.get(sig)
        if skel is None:
            skel = pickle.dumps(copy.deepcopy(value).to("meta"))
            _SKELETONS.clear()
            _SKELETONS[sig] = skel
        return "module", items, skel
    if isinstance(value, dict):
        items = []
        for k, v in value.items():
            if not isinstance(v, torch.Tensor):
                raise TypeError(f"ShareData: dict entry {k!r} is {type(v).__name__}, expected a tensor")
            items.append((str(k), v))
        return "dict", items, b""
    raise TypeError(f"ShareData: cannot share a {type(value).__name__} (tensor, dict of tensors or nn.Module)")


class ShareData:
    """Same surface as the reference's ShareData, device-resident."""

    def __init__(self, name=None, _attach=False):
        L.lib()
        self._name = name or f"/psvo-share-{os.getpid()}-{uuid.uuid4().hex[:12]}"
        fn = L.lib().psvo_share_attach if _attach else L.lib().psvo_share_create
        h = fn(self._name.encode())
        if not h:
            raise L.PsvoError(f"ShareData({self._name}): {L.lib().psvo_last_error().decode(errors='replace')}")
        self._h = ctypes.c_void_p(h)
        self._owner = not _attach
        self._meta_buf = ctypes.create_string_buffer(META_CAP)

    # -- process hand-off: children attach by name -----------------------
    def __reduce__(self):
        return (_attach, (self._name,))

    @property
    def name(self):
        return self._name

    def close(self):
        """Detach (frees this process's published slots); the creator also
        unlinks the segment name."""
        if getattr(self, "_h", None):
            L.lib().psvo_share_detach(self._h)
            self._h = None
            if self._owner:
                L.lib().psvo_share_unlink(self._name.encode())

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- generic channel access ---------------------------------------------
    def publish(self, channel, value):
        """Writer side of a property setter: D2D copy into a free slot."""
        ch = CHANNELS[channel] if isinstance(channel, str) else int(channel)
        kind, items, skel = _flatten(value)
        dev = None
        tensors = []
        for _, t in items:
            t = t.detach()
            if dev is None:
                dev = t.device if t.is_cuda else torch.device("cuda", torch.cuda.current_device())
            tensors.append(t.to(dev).contiguous())   # host tensors (reference setters pass .cpu()) go up once
        entries = [{"name": n, "dtype": str(t.dtype), "shape": list(t.shape)} for (n, _), t in zip(items, tensors)]
        head = json.dumps({"kind": kind, "entries": entries}).encode()
        meta = struct.pack("<I", len(head)) + head + skel
        if len(meta) > META_CAP:
            raise ValueError(f"ShareData: layout of {len(meta)} B exceeds {META_CAP} B")
        n = len(tensors)
        srcs = (ctypes.c_void_p * max(n, 1))(*[t.data_ptr() for t in tensors])
        nbytes = (ctypes.c_int64 * max(n, 1))(*[t.numel() * t.element_size() for t in tensors])
        offsets = (ctypes.c_int64 * max(n, 1))()
        version = ctypes.c_uint64(0)
        with torch.cuda.device(dev if dev is not None else torch.cuda.current_device()):
            st = L.stream_of(dev)
            _check(L.lib().psvo_share_publish(self._h, st, ch, n, srcs, nbytes, meta, len(meta), PUBLISH_TIMEOUT_MS,
                                              offsets, ctypes.byref(version)), "psvo_share_publish")
        return int(version.value)

    def version(self, channel):
        ch = CHANNELS[channel] if isinstance(channel, str) else int(channel)
        return int(L.lib().psvo_share_version(self._h, ch))

    def fetch(self, channel, after=0, device=None, into=None):
        """Reader side: the latest snapshot newer than version `after` as
        (value, version), or None when there is nothing newer.  `into` (a dict
        of tensors or a module from an earlier fetch, same layout) is filled in
        place instead of allocating."""
        ch = CHANNELS[channel] if isinstance(channel, str) else int(channel)
        dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        slot, version = ctypes.c_int(0), ctypes.c_uint64(0)
        meta_len, used, base = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_void_p(0)
        rc = L.lib().psvo_share_acquire(self._h, ch, int(after), ctypes.byref(slot), ctypes.byref(version),
                                        self._meta_buf, META_CAP, ctypes.byref(meta_len), ctypes.byref(used),
                                        ctypes.byref(base))
        if rc < 0:
            _check(-rc, "psvo_share_acquire")
        if rc == 0:
            return None
        try:
            raw = self._meta_buf.raw[:meta_len.value]
            (hl,) = struct.unpack_from("<I", raw)
            head = json.loads(raw[4:4 + hl])
            skel = raw[4 + hl:]
            kind, entries = head["kind"], head["entries"]
            outs = self._targets(kind, entries, skel, dev, into)
            n = len(entries)
            offs, size = [], 0
            for e in entries:  # the writer's 256-B aligned packing (share.cpp publish)
                offs.append(size)
                nb = int(np.prod(e["shape"], dtype=np.int64)) * torch.empty((), dtype=_DTYPES[e["dtype"]]).element_size()
                size += (nb + 255) // 256 * 256
            dsts = (ctypes.c_void_p * max(n, 1))(*[t.data_ptr() for t in outs])
            nbytes = (ctypes.c_int64 * max(n, 1))(*[t.numel() * t.element_size() for t in outs])
            coffs = (ctypes.c_int64 * max(n, 1))(*offs)
            with torch.cuda.device(dev):
                _check(L.lib().psvo_share_read(self._h, L.stream_of(dev), ch, slot.value, n, dsts, coffs, nbytes,
                                               base), "psvo_share_read")
        finally:
            _check(L.lib().psvo_share_release(self._h, ch, slot.value), "psvo_share_release")
        return self._assemble(kind, entries, outs, skel, dev, into), int(version.value)

    @staticmethod
    def _targets(kind, entries, skel, dev, into):
        def fresh(e):
            return torch.empty(e["shape"], dtype=_DTYPES[e["dtype"]], device=dev)

        if into is None:
            return [fresh(e) for e in entries]
        if kind == "module":
            sd = into.state_dict()
            outs = [sd[e["name"]] for e in entries]
        elif kind == "dict":
            outs = [into[e["name"]] for e in entries]
        else:
            outs = [into]
        for t, e in zip(outs, entries):
            if list(t.shape) != e["shape"] or str(t.dtype) != e["dtype"] or not t.is_contiguous():
                raise ValueError(f"ShareData.fetch(into=...): entry {e['name']!r} changed layout")
        return outs

    @staticmethod
    def _assemble(kind, entries, outs, skel, dev, into):
        if into is not None:
            return into
        if kind == "none":
            return None
        if kind == "tensor":
            return outs[0]
        if kind == "dict":
            return {e["name"]: t for e, t in zip(entries, outs)}
        mod = pickle.loads(skel).to_empty(device=dev)   # our own writer's skeleton (meta tensors only)
        mod.load_state_dict(dict(zip((e["name"] for e in entries), outs)), strict=True, assign=True)
        return mod

    def get(self, channel):
        r = self.fetch(channel)
        return None if r is None else r[0]

    # -- reference properties -------------------------------------------
    decoder = property(lambda self: self.get("decoder"), lambda self, v: self.publish("decoder", v))
    points_encoder = property(lambda self: self.get("points_encoder"),
                              lambda self, v: self.publish("points_encoder", v))
    states = property(lambda self: self.get("states"), lambda self, v: self.publish("states", v))
    voxels = property(lambda self: self.get("voxels"), lambda self, v: self.publish("voxels", v))
    octree = property(lambda self: self.get("octree"), lambda self, v: self.publish("octree", v))
    hash_voxel = property(lambda self: self.get("hash_voxel"), lambda self, v: self.publish("hash_voxel", v))

    def _flag(self, i):
        v = L.lib().psvo_share_get_flag(self._h, i)
        if v < 0:
            raise L.PsvoError("psvo_share_get_flag failed")
        return bool(v)

    def _set_flag(self, i, v):
        _check(L.lib().psvo_share_set_flag(self._h, i, int(bool(v))), "psvo_share_set_flag")

    stop_mapping = property(lambda self: self._flag(0), lambda self, v: self._set_flag(0, v))
    stop_tracking = property(lambda self: self._flag(1), lambda self, v: self._set_flag(1, v))

    def push_pose(self, pose):
        """Append a pose (the reference pushes the 3-vector translation,
        tracking.py:159); up to 7 numbers."""
        p = np.ascontiguousarray(np.asarray(pose, dtype=np.float64).reshape(-1))
        _check(L.lib().psvo_share_push_pose(self._h, p.ctypes.data_as(ctypes.c_void_p), int(p.size)),
               "psvo_share_push_pose")

    @property
    def tracking_trajectory(self):
        n = int(L.lib().psvo_share_trajectory(self._h, None, 0))
        buf = np.zeros((max(n, 1), POSE_DIM), dtype=np.float64)
        n = int(L.lib().psvo_share_trajectory(self._h, buf.ctypes.data_as(ctypes.c_void_p), buf.shape[0]))
        return [buf[i, 1:1 + int(buf[i, 0])].copy() for i in range(n)]


def _attach(name):
    return ShareData(name, _attach=True)
