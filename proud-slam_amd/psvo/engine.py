"""Native mapping / tracking iterations (csrc/engine.cpp): one libpsvo call per
bundle_adjust_frames iteration (render_helpers.py:609-672): render_rays →
Criterion → backward → Adam(embeddings).step() + Adam(decoder).step().

Same kernels and numbers as the autograd path (render_rays + Criterion +
loss.backward() + psvo.optim.Adam), without the Python/autograd time between
launches.  Embeddings and decoder parameters are updated in place; the Adam
moments live here (state_dict-compatible with psvo.optim.Adam / torch Adam:
exp_avg / exp_avg_sq / step).
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib as L

_vp, _i32, _i64, _f32, _f64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_double


class MapDesc(ctypes.Structure):
    """Mirror of psvo_map_desc (include/psvo.h)."""
    _fields_ = [("n_nodes", _i64), ("centres", _vp), ("structure", _vp), ("vertex_idx", _vp),
                ("emb", _vp), ("n_emb", _i64), ("emb_m", _vp), ("emb_v", _vp),
                ("dec", _vp * 10), ("dec_m", _vp * 10), ("dec_v", _vp * 10), ("width", _i32),
                ("voxel_size", _f32), ("step_size", _f32), ("max_distance", _f32), ("truncation", _f32),
                ("max_depth", _f32), ("w_rgb", _f32), ("w_depth", _f32), ("w_fs", _f32), ("w_sdf", _f32),
                ("lr_emb", _f64), ("lr_dec", _f64), ("beta1", _f64), ("beta2", _f64), ("eps", _f64),
                ("grad_flat", _vp), ("packed", _vp), ("emb_row_flags", _vp), ("emb_row_local", _vp)]


class MapFrames(ctypes.Structure):
    """Mirror of psvo_map_frames (include/psvo.h)."""
    _fields_ = [("n_frames", _i32), ("rays_per_frame", _i64), ("dirs_cam", _vp), ("poses", _vp), ("pose_m", _vp),
                ("pose_v", _vp), ("pose_step", _vp), ("lr_pose", _f64), ("pose_grad", _vp),
                ("next_dirs_cam", _vp), ("next_seed", ctypes.c_uint64), ("next_stream", _vp),
                ("next_gt_depth", _vp)]


def _lib():
    return L.lib()


class MappingEngine:
    """map_states: psvo.octree.map_states dict (device); decoder: psvo.decoder.Decoder
    (width 128 or 256); criteria: dict of rgb/depth/fs/sdf weights (Criterion args.criteria)."""

    def __init__(self, map_states, decoder, voxel_size, step_size, truncation=0.1, max_distance=10.0,
                 criteria=None, max_depth=10.0, lr_emb=5e-3, lr_dec=5e-3, betas=(0.9, 0.999), eps=1e-8):
        crit = criteria or {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0}
        self.ms = map_states
        self.emb = map_states["voxel_vertex_emb"]
        self.params = decoder.fused_params()
        for t in [self.emb] + self.params:
            if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
                raise RuntimeError("MappingEngine: embeddings / decoder parameters must be contiguous f32 CUDA")
        self.centres = map_states["voxel_center_xyz"].float().contiguous()
        self.structure = map_states["voxel_structure"].int().contiguous()
        self.vertex_idx = map_states["voxel_vertex_idx"].int().contiguous()
        self.emb_m = torch.zeros_like(self.emb)
        self.emb_v = torch.zeros_like(self.emb)
        self.dec_m = [torch.zeros_like(p) for p in self.params]
        self.dec_v = [torch.zeros_like(p) for p in self.params]
        self.step_no = 0
        self.loss_out = torch.empty(16, dtype=torch.float32, device=self.emb.device)
        self.stats = (ctypes.c_int * 16)()
        self.stats_hook = None  # called with the step's statistics after each step_frames (bench accounting)
        # bundle_adjust_frames discards the loss (render_helpers.py:662-676), so its steps skip the value
        # (PSVO_STEP_NO_LOSS); set True to have step_frames return it there too (tests that record it)
        self.ba_loss = os.environ.get("PSVO_BA_LOSS", "0") == "1"
        self._ahead = None  # the camera directions of a queued step_frames look-ahead
        d = MapDesc()
        d.n_nodes = self.centres.shape[0]
        d.centres, d.structure, d.vertex_idx = (t.data_ptr() for t in (self.centres, self.structure,
                                                                        self.vertex_idx))
        d.emb, d.n_emb = self.emb.data_ptr(), self.emb.shape[0]
        d.emb_m, d.emb_v = self.emb_m.data_ptr(), self.emb_v.data_ptr()
        for i in range(10):
            d.dec[i] = self.params[i].data_ptr()
            d.dec_m[i] = self.dec_m[i].data_ptr()
            d.dec_v[i] = self.dec_v[i].data_ptr()
        d.width = decoder.W
        d.voxel_size, d.step_size, d.max_distance, d.truncation = voxel_size, step_size, max_distance, truncation
        d.max_depth = max_depth
        d.w_rgb, d.w_depth = crit["rgb_weight"], crit["depth_weight"]
        d.w_fs, d.w_sdf = crit["fs_weight"], crit["sdf_weight"]
        d.lr_emb, d.lr_dec, d.beta1, d.beta2, d.eps = lr_emb, lr_dec, betas[0], betas[1], eps
        # flat gradient bucket [embeddings | decoder]: what data-parallel ranks all-reduce
        self.grad_flat = torch.zeros(int(_lib().psvo_map_grad_floats_w(self.emb.shape[0], decoder.W)),
                                     dtype=torch.float32, device=self.emb.device)
        d.grad_flat = self.grad_flat.data_ptr()
        self.desc = d
        self.packed = None
        self._tree_key = None   # the map arrays (pointer, shape, version) the packed tree was built from
        self._bound_key = None  # the embedding moments (pointer, version) the row flags were seeded from
        self.refresh_tree()
        # sparse-exact Adam for the embedding table (include/psvo.h emb_row_flags;
        # PSVO_SPARSE_ADAM=0: dense)
        self.row_flags = None
        self.row_local = None  # data parallel: this rank's touched rows (set_exchange)
        if os.environ.get("PSVO_SPARSE_ADAM", "1") != "0":
            self.row_flags = torch.zeros(self.emb.shape[0], dtype=torch.uint8, device=self.emb.device)
            d.emb_row_flags = self.row_flags.data_ptr()
        self._queued = []   # (caller's rays_o, rays_d, seed, converted ro, rd) per queued query
        self.exchange = None
        self.grad_exchange = None
        h = _lib().psvo_engine_new()
        if not h:
            raise L.PsvoError("psvo_engine_new failed")
        self.handle = _vp(h)

    def _map_key(self):
        ms = self.ms
        return tuple((t.data_ptr(), tuple(t.shape), t._version)
                     for t in (ms["voxel_center_xyz"], ms["voxel_structure"], ms["voxel_vertex_idx"]))

    def refresh_tree(self, force=False):
        """(Re)build the breadth-first packed node records the query
        traverses (psvo_pack_tree; same hits as the reference arrays) from the
        current centres / structure — when the map's arrays changed since the
        last build (another tensor, or an in-place write: torch's version
        counter), or with force.  A changed map's arrays are taken again first
        (the engine holds int32 / f32 copies where the caller's dtype differs).
        PSVO_PACKED=0 keeps the reference-array traversal."""
        key = self._map_key()
        if not force and key == self._tree_key:
            return  # unchanged: no 17-level repack on every bundle_adjust_frames call
        if self._tree_key is not None:
            self.centres = self.ms["voxel_center_xyz"].float().contiguous()
            self.structure = self.ms["voxel_structure"].int().contiguous()
            self.vertex_idx = self.ms["voxel_vertex_idx"].int().contiguous()
            d = self.desc
            d.n_nodes = self.centres.shape[0]
            d.centres, d.structure, d.vertex_idx = (t.data_ptr() for t in (self.centres, self.structure,
                                                                            self.vertex_idx))
        self._tree_key = key
        if os.environ.get("PSVO_PACKED", "1") == "0":
            self.packed = None
            self.desc.packed = None
            return
        n = self.centres.shape[0]
        dev = self.centres.device
        if self.packed is None or self.packed.numel() != n * 32:
            self.packed = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        ws = torch.empty(int(_lib().psvo_pack_tree_workspace_ints(n)), dtype=torch.int32, device=dev)
        L.call("psvo_pack_tree", L.stream_of(dev), n, self.centres, self.structure, ws, self.packed)
        self.desc.packed = self.packed.data_ptr()

    def bind_adam(self, emb_m, emb_v, dec_m, dec_v):
        """Use external Adam moments (e.g. the state tensors of the caller's
        torch / psvo Adam optimisers, so that the engine continues their
        state): f32 tensors shaped like the embeddings / fused decoder params."""
        for t, ref in zip([emb_m, emb_v] + list(dec_m) + list(dec_v), [self.emb] * 2 + self.params * 2):
            if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.shape == ref.shape):
                raise RuntimeError("MappingEngine.bind_adam: moments must match the parameters (contiguous f32 CUDA)")
        self.emb_m, self.emb_v, self.dec_m, self.dec_v = emb_m, emb_v, list(dec_m), list(dec_v)
        # rows whose carried-over moments are non-zero are live — unless these are the very moments of the
        # last bind, unwritten by torch since (the engine writes them in place and keeps the flags itself)
        key = (emb_m.data_ptr(), emb_m._version, emb_v.data_ptr(), emb_v._version)
        if self.row_flags is not None and key != self._bound_key:
            L.call("psvo_adam_flags_from_state", L.stream_of(emb_m.device), emb_m.shape[0], emb_m, emb_v,
                   self.row_flags)
        self._bound_key = key
        d = self.desc
        d.emb_m, d.emb_v = emb_m.data_ptr(), emb_v.data_ptr()
        for i in range(10):
            d.dec_m[i] = self.dec_m[i].data_ptr()
            d.dec_v[i] = self.dec_v[i].data_ptr()

    def set_lr(self, lr_emb=None, lr_dec=None):
        if lr_emb is not None:
            self.desc.lr_emb = float(lr_emb)
        if lr_dec is not None:
            self.desc.lr_dec = float(lr_dec)

    def side_wait(self, stream):
        """`stream` (a torch stream) waits for the end of the last step's
        decoder backward (psvo_map_side_wait; a no-op before the first)."""
        L.call("psvo_map_side_wait", self.handle, ctypes.c_void_p(stream.cuda_stream))

    def step_frames(self, dirs_cam, rays_per_frame, poses, pose_m, pose_v, pose_steps, lr_pose, rgb, depth, seed,
                    noise=None, adam_step=None, apply_adam=True, pose_grad=None, next_dirs_cam=None, next_seed=0,
                    next_stream=None, want_loss=True, next_depth=None):
        """One bundle_adjust_frames iteration with keyframe pose updates
        (psvo_map_step_frames): rays from the current poses [F, 6] (frame f
        owns rows [f·rays_per_frame, (f+1)·rays_per_frame) of dirs_cam),
        render + loss + backward, Adam on embeddings / decoder and on every
        pose with pose_steps[f] ≥ 1 (its Adam step number; 0 = fixed pose).
        poses / pose_m / pose_v are updated in place.  Returns the loss
        (want_loss=False: None — the value is not computed, PSVO_STEP_NO_LOSS).
        next_dirs_cam (contiguous f32 [F·rays_per_frame, 3]) / next_seed: the
        next iteration's batch, whose query is queued beside this step's
        weight gradients (the next call must pass exactly that tensor and seed).
        next_stream: the torch stream next_dirs_cam (and the next call's rgb /
        depth) is produced on, if not the current one — only the look-ahead's
        pose step waits for it."""
        if self._queued:
            raise RuntimeError("MappingEngine.step_frames: a query() is queued (rays here come from the poses)")
        if self._ahead is not None and dirs_cam is self._ahead:
            dirs = dirs_cam  # the look-ahead the previous call queued: the same storage
        else:
            dirs = dirs_cam.reshape(-1, 3).float().contiguous()
        if next_dirs_cam is not None:
            if not (next_dirs_cam.is_cuda and next_dirs_cam.dtype == torch.float32 and next_dirs_cam.is_contiguous()
                    and tuple(next_dirs_cam.shape) == tuple(dirs.shape)) or noise is not None:
                raise RuntimeError("MappingEngine.step_frames: next_dirs_cam must be a contiguous f32 [R, 3] "
                                   "device tensor (and no injected noise)")
        n_f = poses.shape[0]
        for t in (poses, pose_m, pose_v):
            if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and tuple(t.shape) == (n_f, 6)):
                raise RuntimeError("MappingEngine.step_frames: poses / moments must be contiguous f32 CUDA [F, 6]")
        if dirs.shape[0] != n_f * int(rays_per_frame):
            raise RuntimeError("MappingEngine.step_frames: dirs_cam must hold F x rays_per_frame rows")
        gt_rgb = rgb.reshape(-1, 3).float().contiguous()
        gt_d = depth.reshape(-1).float().contiguous()
        steps = (ctypes.c_int64 * n_f)(*[int(x) for x in pose_steps])
        fr = MapFrames()
        fr.n_frames, fr.rays_per_frame = n_f, int(rays_per_frame)
        fr.dirs_cam, fr.poses, fr.pose_m, fr.pose_v = dirs.data_ptr(), poses.data_ptr(), pose_m.data_ptr(), \
            pose_v.data_ptr()
        fr.pose_step = ctypes.cast(steps, ctypes.c_void_p)
        fr.lr_pose = float(lr_pose)
        fr.pose_grad = pose_grad.data_ptr() if pose_grad is not None else None
        fr.next_dirs_cam = next_dirs_cam.data_ptr() if next_dirs_cam is not None else None
        fr.next_seed = int(next_seed) & (2 ** 64 - 1)
        fr.next_stream = next_stream.cuda_stream if next_stream is not None else None
        # the next call's GT depths (it must pass this very tensor): the look-ahead's sampler counts the
        # loss normalisers with them (PSVO_STEP_NO_LOSS steps)
        nd = None
        if next_depth is not None and next_dirs_cam is not None:
            nd = next_depth.reshape(-1)
            if not (nd.is_cuda and nd.dtype == torch.float32 and nd.is_contiguous()):
                nd = None
        fr.next_gt_depth = nd.data_ptr() if nd is not None else None
        nz = None
        if noise is not None:
            nz = noise.to(device=dirs.device, dtype=torch.float32).contiguous()
            self._check_noise(nz, dirs, int(rays_per_frame), poses)
        prev_step = self.step_no
        self.step_no = self.step_no + 1 if adam_step is None else int(adam_step)
        rc = _lib().psvo_map_step_frames(self.handle, L.stream_of(dirs.device), ctypes.addressof(self.desc),
                                         ctypes.addressof(fr), gt_rgb.data_ptr(), gt_d.data_ptr(),
                                         nz.data_ptr() if nz is not None else None, int(seed), self.step_no,
                                         (0 if apply_adam else 1) | (0 if want_loss else 4),
                                         self.loss_out.data_ptr(), ctypes.addressof(self.stats))
        if rc != 0:
            # as step(): the failed iteration did not happen — its Adam step number rolls back, and a
            # look-ahead query it may have queued is dropped on the engine side too (the next call's
            # fresh dirs_cam would otherwise be refused against it)
            self.step_no = prev_step
            err = self._error("psvo_map_step_frames", rc)
            try:
                L.call("psvo_map_discard", self.handle)
            except L.PsvoError:
                pass  # a faulted stream: the step's own error is the one to report
            finally:
                self._queued.clear()
                self._ahead = None
            raise err
        self._ahead = next_dirs_cam  # kept alive until the next call consumes its query
        self._ahead_depth = nd
        if self.stats_hook is not None:
            self.stats_hook(self.stats)
        return self.loss_out[0] if want_loss else None

    def _check_noise(self, nz, dirs, rpf, poses):
        """Injected sampler noise must have the layout this batch's sampler
        reads ([200, K', max_steps], voxel_helpers.py:303-328): one synchronous
        intersection of the batch's rays (a test / replay path only)."""
        from .voxel_helpers import _intersect_sorted
        ro = torch.empty_like(dirs)
        rd = torch.empty_like(dirs)
        L.call("psvo_pose_rays_frames", L.stream_of(dirs.device), dirs.shape[0], rpf, poses, dirs, ro, rd)
        d = self.desc
        q = _intersect_sorted(ro, rd, self.centres, self.structure, d.voxel_size, d.max_distance, d.step_size)
        st = q["stats"].cpu()
        P, r_hit, max_ceil = int(st[0]), int(st[1]), int(st[2])
        want = (200, (r_hit + 199) // 200, max_ceil + P)
        if tuple(nz.shape) != want:
            raise ValueError(f"step_frames: noise must be {list(want)} for this batch, got {list(nz.shape)}")

    def set_exchange(self, exchange):
        """Data-parallel mode (psvo.dist.EngineExchange): every step computes
        the loss of the union of all ranks' rays; sum grad_flat over ranks
        (psvo.dist.EngineGradExchange(op="sum")) before adam()."""
        n = int(_lib().psvo_engine_exchange_words(exchange.world, exchange.max_rays_global, exchange.max_rays_rank))
        if n < 0:
            raise ValueError(f"EngineExchange: bad sizes (max_rays_global {exchange.max_rays_global}, "
                             f"max_rays_rank {exchange.max_rays_rank})")
        xi32, xf64 = exchange.buffers(n)
        if xi32.device != self.emb.device:
            raise RuntimeError("EngineExchange buffers must live on the engine's device")
        L.call("psvo_engine_set_exchange", self.handle, exchange.rank, exchange.world, exchange.max_rays_global,
               exchange.max_rays_rank, ctypes.cast(exchange.callback(), _vp), None, xi32, xf64)
        self.exchange = exchange
        if self.row_flags is not None and self.row_local is None:
            # sparse-exact Adam under data parallelism: the step marks this
            # rank's rows here, the gradient exchange marks the union into
            # row_flags (include/psvo.h emb_row_local)
            self.row_local = torch.zeros_like(self.row_flags)
            self.desc.emb_row_local = self.row_local.data_ptr()
        from .dist import EngineGradExchange
        # the union-batch loss: rank gradients add up (on the exchange's group; forced one-rank runs too)
        self.grad_exchange = EngineGradExchange(self, op="sum", group=exchange.group,
                                                force=getattr(exchange, "force", False))

    def _error(self, name, rc):
        msg = _lib().psvo_last_error().decode()
        if self.exchange is not None and self.exchange.error is not None:
            msg += f" ({type(self.exchange.error).__name__}: {self.exchange.error})"
            self.exchange.error = None
        return L.PsvoError(f"{name} failed (code {rc}): {msg}")

    def discard_queued(self):
        """Drop queries queued by query() that no step will consume."""
        L.call("psvo_map_discard", self.handle)
        self._queued.clear()
        self._ahead = None

    def _sync_queue(self):
        """Drop the Python records of queries the engine consumed (a failed
        step consumes its query too)."""
        n = int(_lib().psvo_engine_queued(self.handle))
        while len(self._queued) > n:
            self._queued.pop(0)

    def query(self, rays_o, rays_d, seed):
        """Queue the next iteration's ray query (intersection + sampling) on the
        engine's side stream, so that it overlaps the current step and the next
        step() with the same rays / seed starts without a read-back stall
        (the query reads only the rays and the octree, which the step does not
        change)."""
        ro = rays_o.reshape(-1, 3).float().contiguous()
        rd = rays_d.reshape(-1, 3).float().contiguous()
        rc = _lib().psvo_map_query(self.handle, L.stream_of(ro.device), ctypes.addressof(self.desc), ro.shape[0],
                                   ro.data_ptr(), rd.data_ptr(), int(seed))
        if rc != 0:
            raise self._error("psvo_map_query", rc)
        self._queued.append((rays_o, rays_d, int(seed), ro, rd))   # alive until the consuming step has run

    def step(self, rays_o, rays_d, rgb, depth, seed, apply_adam=True):
        """One iteration; returns the loss (0-dim device tensor, not synchronised;
        the buffer is reused by the next step).  apply_adam=False stops after the
        gradients (self.grad_flat) — all-reduce them, then call adam().  If
        query() queued this batch, its results are used."""
        if self._queued:
            q_o, q_d, q_seed, ro, rd = self._queued[0]
            if q_o is not rays_o or q_d is not rays_d or q_seed != int(seed):
                raise RuntimeError("MappingEngine.step: rays / seed differ from the batch query() queued "
                                   "(pass the same tensor objects and seed)")
        else:
            ro = rays_o.reshape(-1, 3).float().contiguous()
            rd = rays_d.reshape(-1, 3).float().contiguous()
        gt_rgb = rgb.reshape(-1, 3).float().contiguous()
        gt_d = depth.reshape(-1).float().contiguous()
        self.step_no += 1
        rc = _lib().psvo_map_step(self.handle, L.stream_of(ro.device), ctypes.addressof(self.desc), ro.shape[0],
                                  ro.data_ptr(), rd.data_ptr(), gt_rgb.data_ptr(), gt_d.data_ptr(), int(seed),
                                  self.step_no, 0 if apply_adam else 1, self.loss_out.data_ptr(),
                                  ctypes.addressof(self.stats))
        # queued records the engine consumed (the step's kernels are
        # stream-ordered after their last use of the rays)
        self._sync_queue()
        if rc != 0:
            self.step_no -= 1
            raise self._error("psvo_map_step", rc)
        return self.loss_out[0]

    def adam(self):
        """Both Adam steps from self.grad_flat (after a step(apply_adam=False)).
        Data parallel, the embedding step is row-sparse only when this step's
        gradient exchange marked the union of all ranks' rows; otherwise the
        engine steps the table densely (psvo_map_adam_ex, include/psvo.h)."""
        ge = self.grad_exchange
        marked = ge is not None and ge.take_rows_marked()
        L.call("psvo_map_adam_ex", self.handle, L.stream_of(self.emb.device), ctypes.addressof(self.desc),
               self.step_no, 1 if marked else 0)

    PATH_QUERY_SPLIT, PATH_PADDED, PATH_DENSE_DECODER = 1, 2, 4

    def set_paths(self, paths):
        """Run the alternative production kernels on this single-GPU engine
        (cross-checks): PATH_QUERY_SPLIT — the query's statistics / rank pass
        and sample scan as kernels of their own; PATH_PADDED — the padded z
        copy and in-step loss normalisers; PATH_DENSE_DECODER — the width-128
        decoder on every sample instead of the sparse decoder
        (psvo_engine_set_paths)."""
        L.call("psvo_engine_set_paths", self.handle, int(paths))

    def select_stats(self, reset=False):
        """The sparse decoder's sample selection (synchronises): {"kept",
        "composited"} of the last step and their sums over "steps" steps since
        the last reset (psvo_engine_select_stats)."""
        out = (ctypes.c_int64 * 5)()
        L.call("psvo_engine_select_stats", self.handle, L.stream_of(self.emb.device), ctypes.cast(out, ctypes.c_void_p),
               int(bool(reset)))
        return {"kept": out[0], "composited": out[1], "kept_sum": out[2], "composited_sum": out[3], "steps": out[4]}

    def set_timing(self, on):
        """Per-region kernel time (query: intersect / sample / points, interp fwd
        / bwd, decoder fwd / bwd): each kernel a region launches is timed by a
        HIP event pair bound to its own dispatch, a region is the sum of its
        kernels' spans (PSVO_TIMING_MARKERS=1: marker events around the
        region).  on=True: regions serialised on one stream; on="overlap": as
        the untimed step runs them (side streams overlapping the main stream)."""
        L.call("psvo_engine_set_timing", self.handle, 2 if on == "overlap" else int(bool(on)))

    def set_clock(self, max_steps):
        """Record an event on the launching stream at each mapping step's entry
        (up to max_steps; 0: off) — see clock()."""
        L.call("psvo_engine_set_clock", self.handle, int(max_steps))

    def clock(self):
        """(mean GPU-side period per step in ms or None, steps recorded)."""
        ms, n = ctypes.c_double(), ctypes.c_int()
        L.call("psvo_engine_clock", self.handle, ctypes.byref(ms), ctypes.byref(n))
        return (ms.value if ms.value >= 0 else None), n.value

    @staticmethod
    def host_wait_stats(reset=False):
        """(µs the host spent waiting for query statistics, waits, waits that
        found them not yet landed) since the last reset, process-wide."""
        us, calls, waited = ctypes.c_double(), ctypes.c_longlong(), ctypes.c_longlong()
        L.call("psvo_host_wait_stats", ctypes.byref(us), ctypes.byref(calls), ctypes.byref(waited), int(reset))
        return us.value, calls.value, waited.value

    REGIONS = ("mlp_fwd", "mlp_bwd", "interp_fwd", "interp_bwd", "intersect", "sample", "points", "select")

    def timing(self):
        """Mean ms per step of each PSVO_TIME_* region since set_timing(True)."""
        out = (ctypes.c_double * len(self.REGIONS))()
        L.call("psvo_engine_timing", self.handle, ctypes.cast(out, ctypes.c_void_p))
        return dict(zip(self.REGIONS, list(out)))

    @property
    def last_stats(self):
        return list(self.stats)

    def close(self):
        if getattr(self, "handle", None) is not None:
            _lib().psvo_engine_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class TrackingEngine:
    """Native tracking iteration (psvo_track_step): track_frame's loop body
    (render_helpers.py:708-722) — world rays from the pose, render_rays
    against the frozen map, Criterion (weight_depth_loss = the median depth
    filter), backward to the pose only and torch.optim.Adam on the pose — as
    one libpsvo call with a single stats read-back.  The map (map_states) and
    decoder are read, never written."""

    def __init__(self, map_states, decoder, voxel_size, step_size, truncation=0.1, max_distance=10.0,
                 criteria=None, max_depth=10.0, betas=(0.9, 0.999), eps=1e-8):
        crit = criteria or {"rgb_weight": 0.5, "depth_weight": 1.0, "sdf_weight": 5000.0, "fs_weight": 10.0}
        emb = map_states["voxel_vertex_emb"].detach()
        self.params = [p.detach() for p in decoder.fused_params()]
        for t in [emb] + self.params:
            if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
                raise RuntimeError("TrackingEngine: embeddings / decoder parameters must be contiguous f32 CUDA")
        self.dev = emb.device
        self.emb = emb
        self.centres = map_states["voxel_center_xyz"].float().contiguous()
        self.structure = map_states["voxel_structure"].int().contiguous()
        self.vertex_idx = map_states["voxel_vertex_idx"].int().contiguous()
        d = MapDesc()
        d.n_nodes = self.centres.shape[0]
        d.centres, d.structure, d.vertex_idx = (t.data_ptr() for t in (self.centres, self.structure,
                                                                        self.vertex_idx))
        d.emb, d.n_emb = emb.data_ptr(), emb.shape[0]
        for i in range(10):
            d.dec[i] = self.params[i].data_ptr()
        d.width = decoder.W
        d.voxel_size, d.step_size, d.max_distance, d.truncation = voxel_size, step_size, max_distance, truncation
        d.max_depth = max_depth
        d.w_rgb, d.w_depth = crit["rgb_weight"], crit["depth_weight"]
        d.w_fs, d.w_sdf = crit["fs_weight"], crit["sdf_weight"]
        d.beta1, d.beta2, d.eps = betas[0], betas[1], eps
        self.desc = d
        # pose [t | w] and its Adam state; pose_grad / loss of the last step
        self.pose = torch.zeros(6, dtype=torch.float32, device=self.dev)
        self.pose_m = torch.zeros(6, dtype=torch.float32, device=self.dev)
        self.pose_v = torch.zeros(6, dtype=torch.float32, device=self.dev)
        self.pose_grad = torch.zeros(8, dtype=torch.float32, device=self.dev)
        self.loss_out = torch.empty(16, dtype=torch.float32, device=self.dev)
        self.stats = (ctypes.c_int * 16)()
        self.step_no = 0
        h = _lib().psvo_engine_new()
        if not h:
            raise L.PsvoError("psvo_engine_new failed")
        self.handle = _vp(h)

    def reset(self, pose_data):
        """Start a frame from pose parameters [t | w] (a fresh torch.optim.Adam)."""
        self.pose.copy_(torch.as_tensor(pose_data, dtype=torch.float32).reshape(6))
        self.pose_m.zero_()
        self.pose_v.zero_()
        self.step_no = 0

    def step(self, dirs_cam, rgb, depth, seed, lr=1e-3, depth_variance=False, apply_adam=True, noise=None):
        """One iteration on camera-frame directions [R,3] with their gt rgb
        [R,3] / depth [R]; returns the loss (0-dim device tensor, reused).
        noise: the sampler's noise [200, K', max_steps] (as the reference
        draws it; tests), else drawn on the device from `seed`."""
        dirs = dirs_cam.reshape(-1, 3).float().contiguous()
        gt_rgb = rgb.reshape(-1, 3).float().contiguous()
        gt_d = depth.reshape(-1).float().contiguous()
        nz = None
        if noise is not None:
            nz = torch.as_tensor(noise).to(device=self.dev, dtype=torch.float32).contiguous()
            if nz.dim() != 3 or nz.shape[0] != 200 or nz.shape[1] != -(-dirs.shape[0] // 200):
                raise ValueError(f"TrackingEngine.step: noise must be [200, K', max_steps], got {tuple(nz.shape)}")
        self.step_no += 1
        flags = (0 if apply_adam else 1) | (2 if depth_variance else 0)
        rc = _lib().psvo_track_step(self.handle, L.stream_of(self.dev), ctypes.addressof(self.desc), dirs.shape[0],
                                    dirs.data_ptr(), gt_rgb.data_ptr(), gt_d.data_ptr(), self.pose.data_ptr(),
                                    self.pose_m.data_ptr(), self.pose_v.data_ptr(), float(lr),
                                    nz.data_ptr() if nz is not None else None, int(seed), self.step_no, flags,
                                    self.pose_grad.data_ptr(), self.loss_out.data_ptr(), ctypes.addressof(self.stats))
        if rc != 0:
            raise L.PsvoError(f"psvo_track_step failed (code {rc}): {_lib().psvo_last_error().decode()}")
        return self.loss_out[0]

    def track_frame(self, frame_pose, curr_frame, N_rays=512, num_iterations=10, learning_rate=1e-3,
                    depth_variance=False, seed=None, noise=None):
        """track_frame (render_helpers.py:679-761) on the native step: samples
        N_rays pixels per iteration from curr_frame (sample_rays → sample_idx)
        and returns an OptimizablePose holding the optimised parameters.
        noise: a callable iteration → the sampler noise (tests)."""
        from .pose import OptimizablePose
        self.reset(frame_pose.data.detach())
        dirs_all = curr_frame.rays_d.reshape(-1, 3)
        rgb_all = curr_frame.rgb.reshape(-1, 3)
        depth_all = curr_frame.depth.reshape(-1)
        base = int(torch.randint(0, 2 ** 62, (1,)).item()) if seed is None else int(seed)
        for it in range(num_iterations):
            curr_frame.sample_rays(N_rays)
            idx = curr_frame.sample_idx
            self.step(dirs_all.index_select(0, idx), rgb_all.index_select(0, idx), depth_all.index_select(0, idx),
                      base + it, learning_rate, depth_variance, noise=noise(it) if callable(noise) else None)
        return OptimizablePose(self.pose.detach().clone())

    @property
    def last_stats(self):
        return list(self.stats)

    def close(self):
        if getattr(self, "handle", None) is not None:
            _lib().psvo_engine_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
