"""GP terrain mapper on MI355X -- the host-side mirror of the external
``terrain_mapping_node`` that serves ``get_terrain_map_with_uncertainty`` to
the reference node (launch/safe_bayesian_optimization.launch.py:111-117,
hyper-parameters config/lpsc.yaml:35-37, client
src/safe_bayesian_optimization_node.cpp:75-77, request/response :576-644).

Everything numeric runs in libsbo.so (HIP kernels + rocSOLVER); this module
only marshals arrays.  Inputs may be numpy arrays (host) or torch tensors on
the GPU (zero-copy, passed as device pointers).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _native as N
from .terrain import Hyper


def _is_dev(a) -> bool:
    return hasattr(a, "is_cuda") and bool(a.is_cuda)


def _ptr(a):
    if a is None:
        return None
    if _is_dev(a):
        return ctypes.c_void_p(a.data_ptr())
    return ctypes.c_void_p(a.ctypes.data)


def _host(a, dt):
    return np.ascontiguousarray(np.asarray(a), dtype=dt)


def _prep(arrs, dt_np, dt_torch_name):
    """Make every input the same kind: all device (contiguous, right dtype) or all host."""
    if all(_is_dev(a) for a in arrs):
        import torch
        dt = getattr(torch, dt_torch_name)
        return [a.contiguous().to(dt) for a in arrs], N.SBO_DEVICE_PTRS
    if any(_is_dev(a) for a in arrs):
        raise TypeError("mix of device tensors and host arrays")
    return [_host(a, dt_np) for a in arrs], 0


def _to_hyper(h: Hyper) -> N.sbo_hyper:
    return N.sbo_hyper(float(h.length_scale), float(h.sigma_f), float(h.noise_level), float(h.prior_mean))


@dataclass
class TerrainMapResponse:
    """Fields of GetTerrainMapWithUncertainty::Response in the order the node
    reads them (node.cpp:607-644)."""
    success: bool
    message: str
    n_width_cells: int
    n_height_cells: int
    x_coords: np.ndarray = field(default_factory=lambda: np.zeros(0))
    y_coords: np.ndarray = field(default_factory=lambda: np.zeros(0))
    values: np.ndarray = field(default_factory=lambda: np.zeros(0))          # mu
    uncertainties: np.ndarray = field(default_factory=lambda: np.zeros(0))   # sigma


class Context:
    """Owns one sbo_ctx (one per thread, bound to a device)."""

    def __init__(self, device: int = 0):
        self._lib = N.lib()
        h = ctypes.c_void_p()
        N.check(self._lib.sbo_create(int(device), ctypes.byref(h)))
        self.handle = h
        self.device = device
        self._torch_stream = None   # the torch stream the context runs on (set_stream), None: its own

    def set_stream(self, stream) -> None:
        """Bind to a HIP stream (a torch.cuda.Stream, a raw handle int, or None)."""
        raw = getattr(stream, "cuda_stream", stream)
        N.check(self._lib.sbo_set_stream(self.handle, ctypes.c_void_p(raw) if raw else None), self.handle)
        if raw and not hasattr(stream, "cuda_stream"):
            import torch
            stream = torch.cuda.ExternalStream(int(raw), device=f"cuda:{self.device}")
        self._torch_stream = stream if raw else None

    # ------------------------------------------------- frontier, 8(f)1
    def frontier(self, Dx, Dy, safe, width: int, height: int) -> np.ndarray:
        """FindSafetyContourIndices (node.cpp:418-497).  Torch device tensors
        (f64 coordinates, u8 mask) take the device raster; numpy arrays the
        host restatement.  Returns the frontier grid indices (int32, host)."""
        (Dx, Dy), fl = _prep([Dx, Dy], np.float64, "float64")
        safe = safe.contiguous() if _is_dev(safe) else _host(safe, np.uint8)
        m = int(Dx.numel() if _is_dev(Dx) else Dx.size)
        cap = 8 * max(1, int(width)) * max(1, int(height)) + 16
        out = np.empty(cap, np.int32)
        cnt = ctypes.c_int64(0)
        self.check(self._lib.sbo_frontier(self.handle, _ptr(Dx), _ptr(Dy), _ptr(safe), m, int(width), int(height),
                                          ctypes.c_void_p(out.ctypes.data), cap, ctypes.byref(cnt), fl))
        return out[:cnt.value].copy()

    def subgoal(self, Dx, Dy, lo, hi, safe, width: int, height: int, gx: float = 0.0, gy: float = 0.0) -> int:
        """GetNextSubgoal (node.cpp:499-550) on device tensors or host arrays;
        -1 when there is no frontier."""
        (Dx, Dy, lo, hi), fl = _prep([Dx, Dy, lo, hi], np.float64, "float64")
        safe = safe.contiguous() if _is_dev(safe) else _host(safe, np.uint8)
        m = int(Dx.numel() if _is_dev(Dx) else Dx.size)
        idx = ctypes.c_int64(-1)
        self.check(self._lib.sbo_subgoal(self.handle, _ptr(Dx), _ptr(Dy), _ptr(lo), _ptr(hi), _ptr(safe), m,
                                         int(width), int(height), float(gx), float(gy), ctypes.byref(idx), fl))
        return int(idx.value)

    def reduce_keys(self, keys, out=None, *, async_: bool | None = None):
        """Combine n raw 16-byte keys ((n, 2) or (2n,) int64: f64 score bits,
        i64 index) into one (sbo_keys_reduce).  Device tensors stay on the
        device -- the reduction runs on this context's stream -- and the (2,)
        int64 result tensor is returned; host arrays return a (score, index)
        pair.  async_ (default: whenever possible) leaves out the host sync;
        it needs the context bound to a torch stream (set_stream), since torch
        cannot wait on the library's own stream -- async_=True without one
        raises instead of silently blocking."""
        n = int((keys.numel() if _is_dev(keys) else np.asarray(keys).size) // 2)
        if _is_dev(keys):
            import torch
            if async_ and self._torch_stream is None:
                raise ValueError("reduce_keys(async_=True) needs set_stream(): the library's own stream "
                                 "cannot be waited on by torch")
            keys = keys.contiguous()
            if out is None:
                out = torch.empty(2, dtype=torch.int64, device=keys.device)
            fl = N.SBO_DEVICE_PTRS | (N.SBO_ASYNC if async_ is not False else 0)
            # keys / out live on torch's current stream (an all-gather wrote
            # keys there): order the library's stream after it, keep keys
            # alive for the allocator until the reduce ran, and order the
            # current stream after the reduce for whoever reads out
            cur = torch.cuda.current_stream(keys.device)
            lib_s = self._torch_stream
            if lib_s is None:
                # the library's own stream, which torch cannot wait on: sync
                # the current stream before and the library's after (no async)
                cur.synchronize()
                fl = N.SBO_DEVICE_PTRS
            elif lib_s.cuda_stream != cur.cuda_stream:
                lib_s.wait_stream(cur)
            self.check(self._lib.sbo_keys_reduce(self.handle, _ptr(keys), n, _ptr(out), fl))
            if lib_s is not None and lib_s.cuda_stream != cur.cuda_stream:
                keys.record_stream(lib_s)
                out.record_stream(lib_s)
                cur.wait_stream(lib_s)
            return out
        k = np.ascontiguousarray(np.asarray(keys, np.int64).reshape(-1))
        r = N.sbo_key()
        self.check(self._lib.sbo_keys_reduce(self.handle, ctypes.c_void_p(k.ctypes.data), n, ctypes.byref(r), 0))
        return r.score, int(r.idx)

    def close(self) -> None:
        if getattr(self, "handle", None):
            self._lib.sbo_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, status: int) -> None:
        N.check(status, self.handle)


class TerrainMapper:
    """GP posterior over a terrain grid (a1-a4) on one GPU."""

    def __init__(self, device: int = 0, hyper: Hyper | None = None, ctx: Context | None = None):
        self.ctx = ctx or Context(device)
        self.hyper = hyper or Hyper()
        self._lib = N.lib()

    # -------------------------------------------------------------- fitting
    def fit(self, x, y, obs, *, async_: bool = False) -> None:
        (x, y, obs), fl = _prep([x, y, obs], np.float32, "float32")
        if async_:
            fl |= N.SBO_ASYNC
        n = int(x.numel() if _is_dev(x) else x.size)
        self.ctx.check(self._lib.sbo_fit(self.ctx.handle, _ptr(x), _ptr(y), _ptr(obs), n,
                                         _to_hyper(self.hyper), fl))

    def append(self, x, y, obs) -> None:
        (x, y, obs), fl = _prep([x, y, obs], np.float32, "float32")
        b = int(x.numel() if _is_dev(x) else x.size)
        self.ctx.check(self._lib.sbo_append(self.ctx.handle, _ptr(x), _ptr(y), _ptr(obs), b, fl))

    @property
    def n(self) -> int:
        return int(self._lib.sbo_num_train(self.ctx.handle))

    # ----------------------------------------------------------- prediction
    def predict(self, qx, qy, *, out=None, async_: bool = False):
        """Posterior mean and latent std at the queries (f32)."""
        (qx, qy), fl = _prep([qx, qy], np.float32, "float32")
        if async_:
            fl |= N.SBO_ASYNC
        m = int(qx.numel() if _is_dev(qx) else qx.size)
        if out is None:
            if fl & N.SBO_DEVICE_PTRS:
                import torch
                mu = torch.empty(m, dtype=torch.float32, device=qx.device)
                sd = torch.empty_like(mu)
            else:
                mu = np.empty(m, np.float32)
                sd = np.empty(m, np.float32)
        else:
            mu, sd = out
        self.ctx.check(self._lib.sbo_predict(self.ctx.handle, _ptr(qx), _ptr(qy), m, _ptr(mu), _ptr(sd), fl))
        return mu, sd

    def tick(self, qx, qy, beta: float, f_min: float, *, score: int = N.SCORE_WIDTH, index_offset: int = 0,
             outputs: dict | None = None, key_out=None, async_: bool = False):
        """Fused predict -> ComputeSets -> masked argmax (the headline step).

        ``outputs`` may hold preallocated mu/sd/lo/hi/safe arrays (None entries
        are skipped).  Host mode returns an ``sbo_key``; device mode writes the
        16-byte key into ``key_out`` (a device tensor) and returns it."""
        (qx, qy), fl = _prep([qx, qy], np.float32, "float32")
        if async_:
            fl |= N.SBO_ASYNC
        m = int(qx.numel() if _is_dev(qx) else qx.size)
        o = outputs or {}
        if fl & N.SBO_DEVICE_PTRS:
            if key_out is None:
                import torch
                key_out = torch.empty(2, dtype=torch.int64, device=qx.device)
            kp = ctypes.cast(ctypes.c_void_p(key_out.data_ptr()), ctypes.POINTER(N.sbo_key))
            self.ctx.check(self._lib.sbo_tick(self.ctx.handle, _ptr(qx), _ptr(qy), m, float(beta), float(f_min),
                                              int(score), int(index_offset), _ptr(o.get("mu")), _ptr(o.get("sd")),
                                              _ptr(o.get("lo")), _ptr(o.get("hi")), _ptr(o.get("safe")), kp, fl))
            return key_out
        key = N.sbo_key()
        self.ctx.check(self._lib.sbo_tick(self.ctx.handle, _ptr(qx), _ptr(qy), m, float(beta), float(f_min),
                                          int(score), int(index_offset), _ptr(o.get("mu")), _ptr(o.get("sd")),
                                          _ptr(o.get("lo")), _ptr(o.get("hi")), _ptr(o.get("safe")),
                                          ctypes.byref(key), fl))
        return key

    def query_cost(self, qx, qy):
        """Sweep work of each query under the current fit (sbo_query_cost):
        the k-tiles its 128-query block multiplies, per query.  Deterministic,
        so every rank computes the same cost-balanced shard cut
        (dist.balanced_shard_range)."""
        (qx, qy), fl = _prep([qx, qy], np.float32, "float32")
        m = int(qx.numel() if _is_dev(qx) else qx.size)
        if fl & N.SBO_DEVICE_PTRS:
            import torch
            cost = torch.empty(m, dtype=torch.float32, device=qx.device)
        else:
            cost = np.empty(m, np.float32)
        self.ctx.check(self._lib.sbo_query_cost(self.ctx.handle, _ptr(qx), _ptr(qy), m, _ptr(cost), fl))
        return cost

    # --------------------------------------------------------- test access
    def order(self) -> np.ndarray:
        """Caller's training index of each internal row (the factor's order)."""
        o = np.empty(self.n, np.int64)
        self.ctx.check(self._lib.sbo_get_order(self.ctx.handle, _ptr(o)))
        return o

    def bounds(self):
        """((x0, x1), (y0, y1)) of every fitted or appended training point
        (sbo_get_bounds; survives export/import), or None before a fit."""
        b = np.zeros(4, np.float64)
        st = self._lib.sbo_get_bounds(self.ctx.handle, _ptr(b))
        if st == N.SBO_E_STATE:
            return None
        self.ctx.check(st)
        return (float(b[0]), float(b[1])), (float(b[2]), float(b[3]))

    def jitter(self) -> float:
        """Diagonal jitter the current fit needed (SBO_OPT_JITTER_RETRIES; 0.0
        when the first factorization succeeded)."""
        j = ctypes.c_double()
        self.ctx.check(self._lib.sbo_get_jitter(self.ctx.handle, ctypes.byref(j)))
        return j.value

    def skip_info(self):
        """(cutoff exponent L in effect, max_i |A_i|_1, |sf2 alpha|_1)."""
        L, r, a = ctypes.c_int(), ctypes.c_double(), ctypes.c_double()
        self.ctx.check(self._lib.sbo_get_skip(self.ctx.handle, ctypes.byref(L), ctypes.byref(r), ctypes.byref(a)))
        return L.value, r.value, a.value

    def precision(self):
        """(precise sweep in effect, the probe's fast-sweep variance error,
        smallest and largest probe variance) -- sbo_get_precision."""
        p, e, vmin, vmax = ctypes.c_int(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        self.ctx.check(self._lib.sbo_get_precision(self.ctx.handle, ctypes.byref(p), ctypes.byref(e),
                                                   ctypes.byref(vmin), ctypes.byref(vmax)))
        return bool(p.value), e.value, vmin.value, vmax.value

    def probe_info(self) -> dict:
        """The last precision probe in detail (sbo_get_probe): its grid and
        training-location parts, each part's own normwise variance error and
        the combined one the decision used."""
        from ._native import sbo_probe
        p = sbo_probe()
        self.ctx.check(self._lib.sbo_get_probe(self.ctx.handle, ctypes.byref(p)))
        return {f: getattr(p, f) for f, _ in sbo_probe._fields_}

    def inverse_check(self) -> dict:
        """The fit's inverse accuracy guard (sbo_get_inverse_check,
        SBO_OPT_INV_CHECK): its normwise variance effect, whether it fired and
        recomputed the inverse with dgemm products, and its device time."""
        from ._native import sbo_inv_check
        r = sbo_inv_check()
        self.ctx.check(self._lib.sbo_get_inverse_check(self.ctx.handle, ctypes.byref(r)))
        return {f: getattr(r, f) for f, _ in sbo_inv_check._fields_}

    def warmup(self, n_cap: int, m_cap: int) -> None:
        """Load every code object a fit and a tick need and size the
        workspaces for up to n_cap points / m_cap queries (sbo_warmup); the
        mapper is left unfitted."""
        self.ctx.check(self._lib.sbo_warmup(self.ctx.handle, int(n_cap), int(m_cap), _to_hyper(self.hyper)))

    def trim(self) -> None:
        """Release the workspaces kept between calls (sbo_trim)."""
        self.ctx.check(self._lib.sbo_trim(self.ctx.handle))

    def set_option(self, option: int, value: int) -> None:
        self.ctx.check(self._lib.sbo_set_option(self.ctx.handle, int(option), int(value)))

    def export_state(self):
        """The fitted predictive state as a torch uint8 device tensor
        (broadcast it; ``import_state`` on another rank)."""
        import torch
        nb = ctypes.c_int64(0)
        self.ctx.check(self._lib.sbo_state_bytes(self.ctx.handle, ctypes.byref(nb)))
        buf = torch.empty(nb.value, dtype=torch.uint8, device=f"cuda:{self.ctx.device}")
        self.ctx.check(self._lib.sbo_export_state(self.ctx.handle, ctypes.c_void_p(buf.data_ptr()), nb.value))
        return buf

    def import_state(self, buf) -> None:
        """Adopt a state exported by another context (predict-only until the next fit)."""
        self.ctx.check(self._lib.sbo_import_state(self.ctx.handle, ctypes.c_void_p(buf.data_ptr()),
                                                  int(buf.numel())))

    def factor(self):
        """(L, alpha) in the internal training order (see ``order()``):
        L dense lower (row-major numpy f32), alpha f32."""
        n = self.n
        Lcm = np.empty(n * n, np.float32)
        a = np.empty(n, np.float32)
        self.ctx.check(self._lib.sbo_get_factor(self.ctx.handle, _ptr(Lcm), _ptr(a), 0))
        return Lcm.reshape(n, n).T.copy(), a

    def rbf_fill(self, x, y):
        (x, y), fl = _prep([x, y], np.float32, "float32")
        n = int(x.numel() if _is_dev(x) else x.size)
        if fl & N.SBO_DEVICE_PTRS:
            import torch
            K = torch.empty(n * n, dtype=torch.float32, device=x.device)
        else:
            K = np.empty(n * n, np.float32)
        self.ctx.check(self._lib.sbo_rbf_fill(self.ctx.handle, _ptr(x), _ptr(y), n, _to_hyper(self.hyper),
                                              _ptr(K), fl))
        return K.reshape(n, n)

    # ------------------------------------------------------------- service
    def get_terrain_map_with_uncertainty(self, resolution, x_range=None, y_range=None) -> TerrainMapResponse:
        """Serve the node's request (resolution[2] f32, node.cpp:580-581).

        The mapper's grid rule is not in the reference (the service "will
        calculate dimensions from data bounds", :583-586).  Here the grid spans
        the training-data bounds (or the given ranges) with
        n = floor(extent / resolution) + 1 cells per axis, stored row-major
        (y outer, x inner).  Parity of this rule is unpinned."""
        bounds = self.bounds() if self.n else None
        if bounds is None:
            return TerrainMapResponse(False, "no measurements", 0, 0)
        rx, ry = (float(np.float32(r)) for r in resolution)
        if not (rx > 0 and ry > 0):
            return TerrainMapResponse(False, "resolution must be > 0", 0, 0)
        x0, x1 = x_range if x_range is not None else bounds[0]
        y0, y1 = y_range if y_range is not None else bounds[1]
        w = int(np.floor((x1 - x0) / rx)) + 1
        h = int(np.floor((y1 - y0) / ry)) + 1
        gx = x0 + rx * np.arange(w)
        gy = y0 + ry * np.arange(h)
        QY, QX = np.meshgrid(gy, gx, indexing="ij")
        return self.grid_response(QX.reshape(-1), QY.reshape(-1), w, h)

    def grid_response(self, qx, qy, width: int, height: int) -> TerrainMapResponse:
        mu, sd = self.predict(qx, qy)
        return TerrainMapResponse(True, f"{width}x{height} grid, N={self.n}", int(width), int(height),
                                  np.asarray(qx, np.float64), np.asarray(qy, np.float64),
                                  np.asarray(mu), np.asarray(sd))

    def close(self) -> None:
        self.ctx.close()
