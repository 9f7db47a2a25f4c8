"""Parity at the bench's own sizes: C4 (the headline, N = 16384, 1000 x 1000
grid, default sweep = variant 3 at skip budget B = 20) and C5 (the streaming
loop, 50 appends N 1000 -> 8000, 512 x 512 grid), both through the C ABI on
cuda:0 against the fp64 oracle (oracle/sbo_oracle.c).

What is checked (SURVEY.md 8(c) staged contract):
  * full grid, size-independent: sigma in [0, sigma_f]; bitwise determinism of
    the tick; shard invariance of the argmax key; lo/hi/S and the masked
    argmax bit-exact against the oracle's ComputeSets + argmax given the
    device's own mu/sigma (node.cpp:409-416, the 16-byte key of the tick);
  * a sample of >= 2048 grid points: mu and sigma^2 within 1e-5
    normwise-relative of the fp64 oracle given the device factor (L, alpha)
    -- the values node.cpp:641-643 copies into mu_/std_; the end-to-end
    argmax over the sample equals the oracle's unless the oracle's own top-2
    gap is inside the error the contract allows;
  * C5: after every tenth append the tick's key against the oracle given the
    device mu/sigma; at the end the posterior against the oracle given the
    appended factor and against a fresh refit of all 8000 points.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from safe_bayesian_optimization_amd import TerrainMapper, synthetic  # noqa: E402
from safe_bayesian_optimization_amd.dist import combine_keys, key_tensor_to_pairs  # noqa: E402
from safe_bayesian_optimization_amd.terrain import CONFIGS  # noqa: E402

REL_TOL = 1e-5   # north_star: 1e-5 relative fp32, normwise (max|d| / max|ref|)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def f32(a):
    return np.ascontiguousarray(a, np.float32)


def nrel(a, b):
    return float(np.abs(np.asarray(a, np.float64) - b).max() / max(np.abs(b).max(), 1e-30))


def oracle_given_factor(gm, wl, qx, qy):
    L, alpha = gm.factor()
    o = gm.order()
    Lcm = O.colmajor_from_lower(L.astype(np.float64))
    del L
    h = wl.hyper
    return O.predict(Lcm, alpha.astype(np.float64), f32(wl.x)[o], f32(wl.y)[o], f32(qx), f32(qy),
                     h.length_scale, h.sf2, h.prior_mean)


def full_outputs(m, dev):
    return dict(mu=torch.empty(m, dtype=torch.float32, device=dev), sd=torch.empty(m, dtype=torch.float32, device=dev),
                lo=torch.empty(m, dtype=torch.float64, device=dev), hi=torch.empty(m, dtype=torch.float64, device=dev),
                safe=torch.empty(m, dtype=torch.uint8, device=dev))


def host(outs):
    return {k: v.cpu().numpy() for k, v in outs.items()}


def check_sets_and_key(h, key, beta, f_min, index_offset=0):
    """Stage (4) at full size: the tick's lo/hi/S are the oracle's
    ComputeSets of the tick's own mu/sigma, bit for bit, and its key is the
    oracle's masked argmax of the width hi - lo (node.cpp:516)."""
    olo, ohi, osafe = O.compute_sets(h["mu"], h["sd"], beta, f_min)
    assert np.array_equal(h["lo"], olo) and np.array_equal(h["hi"], ohi)
    assert np.array_equal(h["safe"], osafe)
    oidx, oval = O.argmax(ohi - olo, osafe)
    (ks, ki), = key_tensor_to_pairs(key)
    assert ki == (oidx + index_offset if oidx >= 0 else -1), (ki, oidx)
    if oidx >= 0:
        assert ks == oval
    return oidx


def check_sample(gm, wl, h, sel, beta, f_min):
    """Stage (3) on a sample + the end-to-end argmax over the sample."""
    omu, ovar = oracle_given_factor(gm, wl, wl.qx[sel], wl.qy[sel])
    emu = nrel(h["mu"][sel], omu)
    evar = nrel(h["sd"][sel].astype(np.float64) ** 2, ovar)
    # end to end over the sample: the oracle's own sets from its fp64 mu/sigma
    olo, ohi, osafe = O.compute_sets(omu, np.sqrt(np.maximum(ovar, 0.0)), beta, f_min)
    ow = ohi - olo
    oi, _ = O.argmax(ow, osafe)
    gi, _ = O.argmax(h["hi"][sel] - h["lo"][sel], h["safe"][sel])
    # width = 2 beta sigma; |d sigma| <= |d sigma^2| / (2 sigma) with the
    # contract's 1e-5 |sigma^2|_max -> |d width| <= beta * 1e-5 / sigma_min
    # over the candidates; any index whose oracle width is within that of the
    # best may legitimately win.  The safe set can also differ where lo is
    # within |d lo| of f_min.
    sd_o = np.sqrt(np.maximum(ovar, 0.0))
    if gi != oi:
        tol = 4.0 * beta * REL_TOL * max(np.abs(ovar).max(), 1e-30) / max(min(sd_o[oi], sd_o[gi]), 1e-12)
        near_edge = abs(olo[gi] - f_min) < tol or abs(olo[oi] - f_min) < tol
        assert near_edge or abs(ow[oi] - ow[gi]) <= tol, (gi, oi, ow[oi], ow[gi], tol)
    return emu, evar, gi == oi


def test_c4_headline(dev):
    """C4 at the bench's default: N = 16384, 10^6 grid points, variant 3, B = 20."""
    n, gw, gh = CONFIGS["C4"]
    wl = synthetic(n, gw, gh, seed=0, name="C4")
    gm = TerrainMapper(0, wl.hyper)
    t = lambda a: torch.tensor(f32(a), device=dev)  # noqa: E731
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    assert gm.skip_info()[0] > 0   # the budgeted skip is on (the bench path)
    qx, qy = t(wl.qx), t(wl.qy)
    m = qx.numel()
    outs = full_outputs(m, dev)
    k1 = gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs).clone()
    torch.cuda.synchronize()
    h = host(outs)
    # determinism: a second tick is bitwise identical
    outs2 = full_outputs(m, dev)
    k2 = gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs2).clone()
    torch.cuda.synchronize()
    assert torch.equal(k1, k2)
    for name in ("mu", "sd", "lo", "hi", "safe"):
        assert torch.equal(outs[name], outs2[name]), name
    del outs2
    assert np.all(h["sd"] >= 0) and np.all(h["sd"] <= np.sqrt(wl.hyper.sf2) * (1 + 1e-6))
    assert np.all(np.isfinite(h["mu"]))
    # shard invariance: four uneven contiguous strips combine to the same key
    cuts = [0, 131072, 400000, 777777, m]
    keys = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        keys.append(gm.tick(qx[a:b], qy[a:b], wl.beta, wl.f_min, index_offset=a).clone())
    torch.cuda.synchronize()
    assert combine_keys(key_tensor_to_pairs(torch.stack(keys))) == key_tensor_to_pairs(k1)[0]
    check_sets_and_key(h, k1, wl.beta, wl.f_min)
    sel = np.sort(np.random.default_rng(4).choice(m, 3072, replace=False))
    emu, evar, same = check_sample(gm, wl, h, sel, wl.beta, wl.f_min)
    print(f"C4 sample of {sel.size}: mu {emu:.2e} var {evar:.2e} argmax same={same}")
    assert emu < REL_TOL and evar < REL_TOL
    gm.close()


def test_c2_exact_workload(dev):
    """C2 exactly as the bench runs it (BASELINE.json configs[1]): N = 2048,
    the 256 x 256 grid, default options -- the whole grid against the fp64
    oracle given the device factor (cheap at this N), lo/hi/S and the key
    bit-exact, a second tick bitwise identical."""
    n, gw, gh = CONFIGS["C2"]
    wl = synthetic(n, gw, gh, seed=0, name="C2")
    gm = TerrainMapper(0, wl.hyper)
    t = lambda a: torch.tensor(f32(a), device=dev)  # noqa: E731
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    assert not gm.precision()[0]          # the fast sweep, as in the bench line
    qx, qy = t(wl.qx), t(wl.qy)
    m = qx.numel()
    outs = full_outputs(m, dev)
    k1 = gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs).clone()
    outs2 = full_outputs(m, dev)
    k2 = gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs2).clone()
    torch.cuda.synchronize()
    assert torch.equal(k1, k2) and all(torch.equal(outs[k], outs2[k]) for k in outs)
    h = host(outs)
    check_sets_and_key(h, k1, wl.beta, wl.f_min)
    sel = np.arange(m)
    emu, evar, same = check_sample(gm, wl, h, sel, wl.beta, wl.f_min)
    print(f"C2 whole grid ({m}): mu {emu:.2e} var {evar:.2e} argmax same={same}")
    assert emu < REL_TOL and evar < REL_TOL
    gm.close()


def test_c5_streaming_loop(dev):
    """C5: fit 1000 points, 50 appends to 8000, a 512 x 512 tick after each."""
    n_end, n0, iters, g = 8000, 1000, 50, 512
    wl = synthetic(n_end, g, g, seed=0, name="C5")
    chunks = np.linspace(n0, n_end, iters + 1).round().astype(int)
    t = lambda a: torch.tensor(f32(a), device=dev)  # noqa: E731
    X, Y, OBS = t(wl.x), t(wl.y), t(wl.obs)
    qx, qy = t(wl.qx), t(wl.qy)
    m = qx.numel()
    gm = TerrainMapper(0, wl.hyper)
    gm.fit(X[:n0], Y[:n0], OBS[:n0])
    outs = full_outputs(m, dev)
    for i in range(iters):
        gm.append(X[chunks[i]:chunks[i + 1]], Y[chunks[i]:chunks[i + 1]], OBS[chunks[i]:chunks[i + 1]])
        key = gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs).clone()
        if i % 10 == 9 or i == iters - 1:
            torch.cuda.synchronize()
            h = host(outs)
            assert np.all(h["sd"] >= 0) and np.all(h["sd"] <= 1.0 + 1e-6)
            check_sets_and_key(h, key, wl.beta, wl.f_min)
    assert gm.n == n_end
    h = host(outs)
    sel = np.sort(np.random.default_rng(5).choice(m, 4096, replace=False))
    emu, evar, same = check_sample(gm, wl, h, sel, wl.beta, wl.f_min)
    print(f"C5 after 50 appends, sample of {sel.size}: mu {emu:.2e} var {evar:.2e} argmax same={same}")
    assert emu < REL_TOL and evar < REL_TOL
    # against a refit of the same 8000 points (different factorisation order
    # of the same matrix: f32 Cholesky differences, not the contract's 1e-5)
    ref = TerrainMapper(0, wl.hyper, ctx=gm.ctx)
    ref.fit(X, Y, OBS)
    ro = full_outputs(m, dev)
    ref.tick(qx, qy, wl.beta, wl.f_min, outputs=ro)
    torch.cuda.synchronize()
    r = host(ro)
    dm, dv = nrel(h["mu"], r["mu"].astype(np.float64)), nrel(h["sd"].astype(np.float64) ** 2,
                                                             r["sd"].astype(np.float64) ** 2)
    print(f"C5 append vs refit: mu {dm:.2e} var {dv:.2e}")
    assert dm < 1e-4 and dv < 1e-4
    gm.close()


@pytest.mark.parametrize("gw,gh", [(1000, 1000), (300, 120)])
def test_lpsc_stress_box(dev, gw, gh):
    """The mapping node's own domain (config/lpsc.yaml:32-37): N = 16384 on
    x [0, 1] x y [0, 2.5], l = 0.4, sigma_f = 1, noise 0.1 -- the bench's
    stress regime -- on the bench's 1000 x 1000 grid and on the mapper's own
    resolution [300, 120] grid, default options.  The variance is 2e-4..3e-3
    there (dense data), so sigma^2 = sf2 - |V|^2 cancels almost all of |V|^2:
    the fast split sweep is 5e-4 off the oracle (an f32 strtrs on the same
    factor 7e-5).  The fit-time probe must select the precise f64 sweep, and
    mu and sigma^2 must meet the 1e-5 contract on a 3072-point sample against
    the fp64 oracle given the device factor; lo/hi/S and the key bit-exact."""
    from safe_bayesian_optimization_amd import _native as N
    from safe_bayesian_optimization_amd.terrain import synthetic_box
    wl = synthetic_box(16384, gw, gh, seed=0)
    gm = TerrainMapper(0, wl.hyper)
    t = lambda a: torch.tensor(f32(a), device=dev)  # noqa: E731
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    precise, perr, vmin, vmax = gm.precision()
    print(f"lpsc box {gw}x{gh}: precise={precise}, fast sweep's probe error {perr:.2e}, probe var {vmin:.2e}..{vmax:.2e}")
    assert precise and perr > 1e-5
    qx, qy = t(wl.qx), t(wl.qy)
    m = qx.numel()
    outs = full_outputs(m, dev)
    k1 = gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs).clone()
    torch.cuda.synchronize()
    h = host(outs)
    assert np.all(h["sd"] >= 0) and np.all(h["sd"] <= 1.0 + 1e-6)
    check_sets_and_key(h, k1, wl.beta, wl.f_min)
    sel = np.sort(np.random.default_rng(6).choice(m, min(3072, m), replace=False))
    emu, evar, same = check_sample(gm, wl, h, sel, wl.beta, wl.f_min)
    # the fast sweep on the same sample, for the record
    gm.set_option(N.SBO_OPT_PRECISION, 0)
    of = full_outputs(m, dev)
    gm.tick(qx, qy, wl.beta, wl.f_min, outputs=of)
    torch.cuda.synchronize()
    omu, ovar = oracle_given_factor(gm, wl, wl.qx[sel], wl.qy[sel])
    fvar = nrel(of["sd"].cpu().numpy()[sel].astype(np.float64) ** 2, ovar)
    fmu = nrel(of["mu"].cpu().numpy()[sel], omu)
    print(f"lpsc box {gw}x{gh}, sample of {sel.size}: precise mu {emu:.2e} var {evar:.2e} argmax same={same}; "
          f"fast mu {fmu:.2e} var {fvar:.2e}")
    assert emu < REL_TOL and evar < REL_TOL
    gm.close()


def test_c4_bitwise_across_sweep_groups(dev):
    """The split sweep's staging (LDS-DMA stages, the step-record windows and
    their refills) at C4 size: the default tick with the persistent sweep cut
    into 256 (one per CU), 200, 97 and 31 workgroup ranges -- every range
    starts and ends at other items, so window boundaries fall at other steps
    -- must give bitwise the same mu, sigma and key (a reverted
    one-step variant once differed in 20 of 10^6 sigma; this pins the shared
    staging code at the bench's own size)."""
    from safe_bayesian_optimization_amd import _native as N
    n, gw, gh = CONFIGS["C4"]
    wl = synthetic(n, gw, gh, seed=0, name="C4")
    gm = TerrainMapper(0, wl.hyper)
    t = lambda a: torch.tensor(f32(a), device=dev)  # noqa: E731
    gm.fit(t(wl.x), t(wl.y), t(wl.obs))
    qx, qy = t(wl.qx), t(wl.qy)
    m = qx.numel()
    ref = None
    try:
        for groups in (0, 200, 97, 31):
            gm.set_option(N.SBO_OPT_SWEEP_GROUPS, groups)
            outs = full_outputs(m, dev)
            k = gm.tick(qx, qy, wl.beta, wl.f_min, outputs=outs).clone()
            torch.cuda.synchronize()
            if ref is None:
                ref = (k, outs)
                continue
            assert torch.equal(k, ref[0]), groups
            for name in ("mu", "sd"):
                diff = int((outs[name] != ref[1][name]).sum())
                assert diff == 0, (groups, name, diff)
    finally:
        gm.set_option(N.SBO_OPT_SWEEP_GROUPS, 0)
    gm.close()
