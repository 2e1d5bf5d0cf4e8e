"""gt:mi355x parity on the GPU: every golden case, plus full-size hot-path configs vs the C oracle.

Small cases compare against the reference numpy-backend golden vectors (bit-exact unless the
case states a tolerance: transcendental functions differ by ULPs between glibc and ocml).
Full-size cases (BASELINE.json configs C2-C4) compare against the C oracle bit-exactly.
"""

import numpy as np
import pytest

import golden_utils as gu
import stencil_cases as sc

pytestmark = pytest.mark.gpu

BACKEND = "gt:mi355x"


def _torch():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch


def _origin_of(case, name, ndim):
    o = case.origin
    if o is None:
        return (0,) * ndim
    if isinstance(o, dict):
        return tuple(o.get(name, o.get("_all_", (0,) * ndim)))[:ndim]
    return tuple(o)[:ndim]


def run_case_on_gpu(case, opts=None, tune=0):
    """Run a golden case through gt:mi355x; ``tune`` > 0 first re-homes the written fields with
    ``storage.placement.tune_written_fields`` (that many candidate buffer sets)."""
    from gt4py_amd import gtscript, storage

    stencil = gtscript.stencil(backend=BACKEND, definition=case.definition, externals=case.externals,
                               name=f"gpu.{case.name}", **(opts or {}))
    host = case.make_inputs()
    dev = {}
    for k, v in host.items():
        if v is None:
            dev[k] = None
            continue
        fi = stencil.field_info.get(k)
        if fi is None:  # unused by the stencil: any layout
            dev[k] = storage.from_array(v, None, backend=BACKEND, aligned_index=_origin_of(case, k, v.ndim))
            continue
        axes = tuple(fi.axes)
        dims = axes + tuple(str(d) for d in range(len(fi.data_dims)))
        o = case.origin
        if isinstance(o, dict):
            org = tuple(o.get(k, o.get("_all_", (0,) * len(axes))))[: len(axes)]
        elif o is None:
            org = (0,) * len(axes)
        else:
            org = tuple(o["IJK".index(a)] for a in axes)
        dev[k] = storage.from_array(
            v, None, backend=BACKEND, aligned_index=org + (0,) * len(fi.data_dims), dimensions=dims
        )
    kw = {}
    if case.origin is not None:
        kw["origin"] = case.origin
    if case.domain is not None:
        kw["domain"] = case.domain
    if tune:
        from gt4py_amd.storage.placement import tune_written_fields

        before = {k: storage.to_numpy(v) for k, v in dev.items() if v is not None}
        stencil(**dev, **case.params, **kw)  # validate once (the tuner's calls skip validation)
        import torch

        for k, v in before.items():  # undo that call: the case's expected outputs start from the inputs
            dev[k].copy_(torch.from_numpy(np.ascontiguousarray(v)).to(dev[k].device))
        arrays = {k: v for k, v in dev.items() if k in stencil.field_info and v is not None}
        tuned, rep = tune_written_fields(stencil, arrays, params=case.params, candidates=tune, reps=2, **kw)
        assert rep["written"] and len(rep["candidates_ms"]) == tune + 1, rep
        for k, v in before.items():  # the tuner keeps every field's contents, and the caller's arrays'
            gu.assert_match(storage.to_numpy(tuned.get(k, dev[k])), v, name=f"{case.name}:{k} kept")
            gu.assert_match(storage.to_numpy(dev[k]), v, name=f"{case.name}:{k} original restored")
        dev.update(tuned)
    stencil(**dev, **case.params, **kw)
    return {k: (None if v is None else storage.to_numpy(v)) for k, v in dev.items()}


@pytest.mark.parametrize("name", gu.available())
def test_golden_case(name):
    _torch()
    case = sc.CASES[name]
    _, outputs, _ = gu.load(name)
    res = run_case_on_gpu(case)
    for k, v in outputs.items():
        gu.assert_match(res[k], v, rtol=case.rtol, atol=case.atol, name=f"{name}:{k}")


# column-kernel schedules: the two register bands the auto rule (kreg=-1) selects, forced onto every
# case (96 levels, prefetch ring + 2; 48 levels, prefetch 6), no register band, no LDS tail, a
# prefetch distance longer than the band (the writer's prologue carries the reader's first levels),
# and both ends of the writer's sweep on chip (ktail_head), with and without a register band
COLUMN_OPT_CASES = ["kcache_forward_backward", "section_gap_register_temp", "tail_bwd_fwd", "tail_bwd_fwd_short",
                    "tail_fwd_bwd_offsets", "tridiag", "tridiag_k161", "tridiag_k2", "tridiag_k70",
                    "tridiag_subdomain_k70", "vertical_advection_dycore", "vertical_advection_dycore_k80",
                    "vertical_advection_dycore_k160", "band_ij_accumulator", "band_ij_accumulator_reader"]
COLUMN_OPTS = [{"kreg": 96}, {"kreg": 48, "kreg_pf": 6}, {"kreg": 0}, {"ktail_lds": 0}, {"kreg": 40, "kreg_pf": 50},
               {"ktail_head": 1}, {"ktail_head": 0}, {"ktail_head": 1, "kreg": 0}, {"ktail_head": 1, "kreg": 40, "kreg_pf": 50}]


@pytest.mark.parametrize("opts", COLUMN_OPTS, ids=lambda o: "_".join(f"{k}{v}" for k, v in o.items()))
@pytest.mark.parametrize("name", COLUMN_OPT_CASES)
def test_golden_column_options(name, opts):
    _torch()
    case = sc.CASES[name]
    _, outputs, _ = gu.load(name)
    res = run_case_on_gpu(case, opts)
    for k, v in outputs.items():
        gu.assert_match(res[k], v, rtol=case.rtol, atol=case.atol, name=f"{name}{opts}:{k}")


# ---------------------------------------------------------------------------------------
# full-size hot-path configurations (BASELINE.json configs) against the C oracle
# ---------------------------------------------------------------------------------------


def _alloc_fill(shape, dtype, rng, lo, hi, origin):
    from gt4py_amd import storage

    host = rng.uniform(lo, hi, size=shape).astype(dtype)
    return host, storage.from_array(host, None, backend=BACKEND, aligned_index=origin)


@pytest.mark.parametrize(
    "dtype,ni,nj,nk",
    # C3 (BASELINE configs[2]); an f32 cast-tree case; C5's per-GPU weak-scaling tile 8192x1024x160 f32
    [(np.float64, 2048, 2048, 160), (np.float32, 1024, 1024, 64), (np.float32, 8192, 1024, 160)],
)
def test_hdiff_full_size_vs_c_oracle(dtype, ni, nj, nk):
    _torch()
    from gt4py_amd import gtscript, storage
    from oracle import c_oracle

    fn = sc.hdiff_f64 if dtype == np.float64 else sc.hdiff_f32
    stencil = gtscript.stencil(backend=BACKEND, definition=fn, name=f"full.hdiff_{np.dtype(dtype).name}")
    rng = np.random.default_rng(1337)
    h = 2
    in_h, in_d = _alloc_fill((ni + 2 * h, nj + 2 * h, nk), dtype, rng, -10, 10, (h, h, 0))
    co_h, co_d = _alloc_fill((ni, nj, nk), dtype, rng, 0, 0.5, (0, 0, 0))
    out_d = storage.zeros((ni, nj, nk), dtype, backend=BACKEND)
    stencil(in_d, out_d, co_d, origin={"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)},
            domain=(ni, nj, nk))
    got = storage.to_numpy(out_d)
    ref = np.zeros((ni, nj, nk), dtype=dtype, order="F")
    org = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    c_oracle.horizontal_diffusion(np.asfortranarray(in_h), ref, np.asfortranarray(co_h), org, (ni, nj, nk))
    gu.assert_match(got, ref, name="hdiff_full")


def test_lap5_full_size_vs_c_oracle():
    _torch()
    from gt4py_amd import gtscript, storage
    from oracle import c_oracle

    ni, nj, nk = 1024, 1024, 80
    stencil = gtscript.stencil(backend=BACKEND, definition=sc.lap5, name="full.lap5")
    rng = np.random.default_rng(1337)
    in_h, in_d = _alloc_fill((ni + 2, nj + 2, nk), np.float64, rng, -10, 10, (1, 1, 0))
    out_d = storage.zeros((ni, nj, nk), np.float64, backend=BACKEND)
    stencil(in_d, out_d, origin={"in_field": (1, 1, 0), "out_field": (0, 0, 0)}, domain=(ni, nj, nk))
    ref = np.zeros((ni, nj, nk), order="F")
    c_oracle.lap5(np.asfortranarray(in_h), ref, {"in_field": (1, 1, 0), "out_field": (0, 0, 0)}, (ni, nj, nk))
    gu.assert_match(storage.to_numpy(out_d), ref, name="lap5_full")


def test_tridiag_full_size_vs_c_oracle():
    _torch()
    from gt4py_amd import gtscript, storage
    from oracle import c_oracle

    ni, nj, nk = 1024, 1024, 160
    stencil = gtscript.stencil(backend=BACKEND, definition=sc.tridiagonal_solver, name="full.tridiag")
    rng = np.random.default_rng(1337)
    hosts, devs = {}, {}
    for name, lo, hi in (("inf", -1, 1), ("diag", 4, 5), ("sup", -1, 1), ("rhs", -10, 10)):
        hosts[name], devs[name] = _alloc_fill((ni, nj, nk), np.float64, rng, lo, hi, (0, 0, 0))
    hosts["out"] = np.zeros((ni, nj, nk))
    devs["out"] = storage.zeros((ni, nj, nk), np.float64, backend=BACKEND)
    stencil(**devs)
    ref = {k: np.asfortranarray(v) for k, v in hosts.items()}
    org = {k: (0, 0, 0) for k in ref}
    c_oracle.tridiagonal_solver(ref["inf"], ref["diag"], ref["sup"], ref["rhs"], ref["out"], org, (ni, nj, nk))
    for k in ("sup", "rhs", "out"):
        gu.assert_match(storage.to_numpy(devs[k]), ref[k], name=f"tridiag_full:{k}")


RAGGED_CHUNK_OPTS = [
    {"jchunk": 4, "jmirror": 1},
    {"jchunk": 8, "jmirror": 1},
    {"jchunk": 8, "jmirror": 0},
    # row_unroll: U copies of the row step per trip, each leaving on its own bound check
    {"jchunk": 8, "jmirror": 1, "row_unroll": 4},
    {"jchunk": 4, "jmirror": 0, "row_unroll": 3},
]


def ragged_chunk_stencil(opts):
    from gt4py_amd import gtscript

    return gtscript.stencil(backend=BACKEND, definition=sc.hdiff_f64, name="gpu.hdiff_ragged", **opts)


@pytest.mark.parametrize("opts", RAGGED_CHUNK_OPTS, ids=lambda o: f"jc{o['jchunk']}_m{o['jmirror']}_u{o.get('row_unroll', 0)}")
@pytest.mark.parametrize("nj", [1, 3, 21, 22, 23, 37])
def test_hdiff_ragged_j_chunks_vs_c_oracle(opts, nj):
    """Odd J chunks stream top-down (jmirror): last chunks of every length, both directions."""
    _torch()
    from gt4py_amd import storage
    from oracle import c_oracle

    ni, nk, h = 150, 3, 2
    stencil = ragged_chunk_stencil(opts)
    rng = np.random.default_rng(nj)
    in_h, in_d = _alloc_fill((ni + 2 * h, nj + 2 * h, nk), np.float64, rng, -10, 10, (h, h, 0))
    co_h, co_d = _alloc_fill((ni, nj, nk), np.float64, rng, 0, 0.5, (0, 0, 0))
    out_d = storage.zeros((ni, nj, nk), np.float64, backend=BACKEND)
    org = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    stencil(in_d, out_d, co_d, origin=org, domain=(ni, nj, nk))
    ref = np.zeros((ni, nj, nk), order="F")
    c_oracle.horizontal_diffusion(np.asfortranarray(in_h), ref, np.asfortranarray(co_h), org, (ni, nj, nk))
    gu.assert_match(storage.to_numpy(out_d), ref, name=f"hdiff_ragged_nj{nj}")


BUFLD_OPTS = [
    {"bufld": 1, "jchunk": 8},
    {"bufld": 1, "jchunk": 4, "jmirror": 0},
    {"bufld": 1, "jchunk": 8, "prefetch": 3},
    {"bufld": 1, "jchunk": 16, "prefetch": 1},
]


def bufld_stencil(dtype, opts):
    from gt4py_amd import gtscript

    defn = sc.hdiff_f64 if dtype == np.float64 else sc.hdiff_f32
    return gtscript.stencil(backend=BACKEND, definition=defn, name="gpu.hdiff_bufld", **opts)


@pytest.mark.parametrize("opts", BUFLD_OPTS, ids=lambda o: "_".join(f"{k}{v}" for k, v in o.items()))
@pytest.mark.parametrize("dtype", [np.float64, np.float32], ids=["f64", "f32"])
@pytest.mark.parametrize("ni,nj", [(150, 22), (1000, 37), (999, 1), (1111, 23)])
def test_hdiff_bufld_strips_vs_c_oracle(opts, dtype, ni, nj):
    """Plane kernels with buffer-descriptor row loads (bufld): interior strips take the branch-free
    slot-ring loop, the first / last strip the clamped one; rows of every chunk length, both J
    directions, several prefetch depths; cells outside the domain keep their sentinel."""
    _torch()
    from gt4py_amd import storage
    from oracle import c_oracle

    nk, h = 3, 2
    stencil = bufld_stencil(dtype, opts)
    rng = np.random.default_rng(ni + nj)
    in_h, in_d = _alloc_fill((ni + 2 * h, nj + 2 * h, nk), dtype, rng, -10, 10, (h, h, 0))
    co_h, co_d = _alloc_fill((ni, nj, nk), dtype, rng, 0, 0.5, (0, 0, 0))
    out_d = storage.full((ni + 3, nj + 2, nk), -7.0, dtype, backend=BACKEND, aligned_index=(1, 1, 0))
    org = {"in_field": (h, h, 0), "out_field": (1, 1, 0), "coeff": (0, 0, 0)}
    stencil(in_d, out_d, co_d, origin=org, domain=(ni, nj, nk))
    ref = np.full((ni + 3, nj + 2, nk), -7.0, dtype=dtype, order="F")
    c_oracle.horizontal_diffusion(np.asfortranarray(in_h), ref, np.asfortranarray(co_h), org, (ni, nj, nk))
    gu.assert_match(storage.to_numpy(out_d), ref, name=f"hdiff_bufld_{ni}x{nj}")


def test_vadv_register_band_vs_numpy_backend():
    """vadv with the default column kernel (auto register band of 96 levels, band
    fronts prefetched; LDS tail below it; scratch for the rest) over several ragged column blocks,
    bit-exact against the numpy backend (itself pinned to the reference goldens), plus the short
    column (nk < the band's minimum) that runs the same library without the band."""
    _torch()
    import bench
    from gt4py_amd import gtscript, storage

    defn = bench.stencil_defs()[("vertical_advection_dycore", np.float64)]
    ext = bench.EXTERNALS["vertical_advection_dycore"]
    gpu = gtscript.stencil(backend=BACKEND, definition=defn, name="parity.vadv_band", externals=ext)
    assert "regband" in gpu._gt_run_impl_.compiled.source
    cpu = gtscript.stencil(backend="numpy", definition=defn, name="parity.vadv_band.np", externals=ext)
    for ni, nj, nk in ((133, 37, 160), (70, 9, 96)):
        rng = np.random.default_rng(ni + nk)
        host = {n: rng.uniform(-1, 1, (ni, nj, nk)) for n in ("utens_stage", "u_stage", "u_pos", "utens")}
        host["wcon"] = rng.uniform(-1, 1, (ni + 1, nj, nk + 1))
        ref = {k: v.copy() for k, v in host.items()}
        cpu(**ref, dtr_stage=0.15, origin=(0, 0, 0), domain=(ni, nj, nk))
        dev = {k: storage.from_array(v, backend=BACKEND) for k, v in host.items()}
        gpu(**dev, dtr_stage=0.15, origin=(0, 0, 0), domain=(ni, nj, nk))
        gu.assert_match(storage.to_numpy(dev["utens_stage"]), ref["utens_stage"], name=f"vadv {ni}x{nj}x{nk}")


def test_outside_domain_untouched():
    """Outputs are written inside the compute domain only (stencil_object.py contract)."""
    torch = _torch()
    from gt4py_amd import gtscript, storage

    stencil = gtscript.stencil(backend=BACKEND, definition=sc.copy_stencil, name="gpu.copy_untouched")
    a = storage.from_array(np.arange(10 * 9 * 7, dtype=np.float64).reshape(10, 9, 7), backend=BACKEND)
    b = storage.full((10, 9, 7), -1.0, backend=BACKEND)
    stencil(a, b, origin=(2, 3, 1), domain=(5, 4, 3))
    bh = storage.to_numpy(b)
    ah = storage.to_numpy(a)
    mask = np.zeros_like(bh, dtype=bool)
    mask[2:7, 3:7, 1:4] = True
    assert (bh[mask] == ah[mask]).all()
    assert (bh[~mask] == -1.0).all()
    del torch


@pytest.mark.parametrize("name", ["hdiff_f64", "hdiff_f32", "suite_hdiff_weight", "multi_stage_temps", "lap5"])
def test_scalar_fallback_layouts(name):
    """K-contiguous (C-order) device tensors have sI != 1: the V=1 plane kernel must run and agree."""
    torch = _torch()
    from gt4py_amd import gtscript, storage

    case = sc.CASES[name]
    _, outputs, _ = gu.load(name)
    stencil = gtscript.stencil(backend=BACKEND, definition=case.definition, externals=case.externals,
                               name=f"gpu.{case.name}")
    host = case.make_inputs()
    dev = {k: (None if v is None else torch.from_numpy(np.ascontiguousarray(v)).cuda()) for k, v in host.items()}
    kw = {}
    if case.origin is not None:
        kw["origin"] = case.origin
    if case.domain is not None:
        kw["domain"] = case.domain
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        stencil(**dev, **case.params, **kw)
    for k, v in outputs.items():
        gu.assert_match(storage.to_numpy(dev[k]), v, rtol=case.rtol, atol=case.atol, name=f"{name}:{k}")


def test_packed_argument_cache_tracks_tensors():
    """Re-allocated tensors (possibly at a recycled id) never reuse a stale packed pointer."""
    _torch()
    from gt4py_amd import gtscript, storage

    st = gtscript.stencil(backend=BACKEND, definition=sc.copy_stencil, name="gpu.pack_cache")
    keep = []
    for trial in range(6):
        a = storage.from_array(np.full((8, 6, 4), float(trial)), backend=BACKEND)
        b = storage.zeros((8, 6, 4), np.float64, backend=BACKEND)
        st(a, b, origin=(0, 0, 0), domain=(8, 6, 4))
        assert (storage.to_numpy(b) == trial).all()
        if trial % 2:
            keep.append((a, b))  # alternate between fresh and surviving objects
        del a, b
    for trial, (a, b) in enumerate(keep):
        a.fill_(100.0 + trial)
        st(a, b, origin=(0, 0, 0), domain=(8, 6, 4), validate_args=False)
        assert (storage.to_numpy(b) == 100.0 + trial).all()


def test_stencil_graph_replay_matches_eager():
    """A captured HIP graph of a stencil sequence replays the same kernels on updated inputs."""
    torch = _torch()
    from gt4py_amd import gtscript, storage
    from gt4py_amd.runtime.graph import StencilGraph

    hd = gtscript.stencil(backend=BACKEND, definition=sc.hdiff_f64, name="gpu.graph.hdiff", device_sync=False)
    cp = gtscript.stencil(backend=BACKEND, definition=sc.copy_stencil, name="gpu.graph.copy", device_sync=False)
    rng = np.random.default_rng(4)
    ni, nj, nk, h = 40, 24, 6, 2
    host_in = rng.uniform(-5, 5, (ni + 2 * h, nj + 2 * h, nk))
    fin = storage.from_array(host_in, backend=BACKEND, aligned_index=(h, h, 0))
    coeff = storage.from_array(rng.uniform(0, 0.5, (ni, nj, nk)), backend=BACKEND)
    out = storage.zeros((ni, nj, nk), np.float64, backend=BACKEND)
    out2 = storage.zeros((ni, nj, nk), np.float64, backend=BACKEND)
    origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}

    def step():
        hd(fin, out, coeff, origin=origin, domain=(ni, nj, nk), validate_args=False)
        cp(out, out2, origin=(0, 0, 0), domain=(ni, nj, nk), validate_args=False)

    g = StencilGraph(step)
    for trial in range(3):
        new_in = rng.uniform(-5, 5, host_in.shape)
        fin.copy_(torch.from_numpy(new_in).to(fin.device))  # in place: the graph re-reads it
        g.replay(sync=True)
        from oracle import numpy_oracle as no  # test infrastructure: the checker

        ref = np.zeros((ni, nj, nk))
        no.horizontal_diffusion(new_in, ref, storage.to_numpy(coeff), origin, (ni, nj, nk))
        got = storage.to_numpy(out2)
        # eager call on the same inputs must agree bit-for-bit with the replay
        out_e = storage.zeros((ni, nj, nk), np.float64, backend=BACKEND)
        hd(fin, out_e, coeff, origin=origin, domain=(ni, nj, nk), validate_args=False)
        torch.cuda.synchronize()
        assert np.array_equal(got, storage.to_numpy(out_e)), trial
        assert np.array_equal(got, ref), trial


def test_batched_halo_copy_more_than_64_faces():
    """More faces than one launch carries (e.g. > 8 fields with the diagonal 2-D scheme): the
    copy is split into launches of at most 64 faces, all on the same stream."""
    torch = _torch()
    from gt4py_amd.distributed.halo_copy import MAX_BOXES, BatchedCopy

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    fields = [torch.rand((19, 11, 3), generator=g, device=dev, dtype=torch.float64) for _ in range(9)]
    boxes = []
    for t in fields:  # 8 faces per field, as the diagonal scheme sends: 72 > 64
        for q in range(8):
            boxes.append((t, (q, q % 5, 0), (2 + q, 2, 3)))
    assert len(boxes) > MAX_BOXES
    bufs = [torch.empty(e[0] * e[1] * e[2], dtype=t.dtype, device=dev) for t, _, e in boxes]
    bc = BatchedCopy([(t, s, e, buf) for (t, s, e), buf in zip(boxes, bufs)])
    assert len(bc.parts) == 2
    bc.run(0)
    torch.cuda.synchronize()
    for (t, s, e), buf in zip(boxes, bufs):
        ref = t[s[0]:s[0] + e[0], s[1]:s[1] + e[1], s[2]:s[2] + e[2]].permute(2, 1, 0).reshape(-1)
        assert torch.equal(buf, ref)


def test_batched_halo_copy_roundtrip():
    """gtmi_halo_copy packs strided boxes of several fields into contiguous buffers and back."""
    torch = _torch()
    from gt4py_amd.distributed.halo_copy import BatchedCopy

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(2)
    a = torch.rand((37, 29, 7), generator=g, device=dev, dtype=torch.float64)
    b = torch.as_strided(torch.rand(40 * 33 * 9, generator=g, device=dev, dtype=torch.float32).contiguous(),
                         (33, 29, 9), (1, 40, 40 * 29))
    boxes = [(a, (0, 3, 0), (37, 2, 7)), (a, (5, 20, 2), (9, 4, 5)), (b, (1, 0, 0), (32, 29, 9))]
    bufs = [torch.empty(e[0] * e[1] * e[2], dtype=t.dtype, device=dev) for t, _, e in boxes]
    BatchedCopy([(t, s, e, buf) for (t, s, e), buf in zip(boxes, bufs)]).run(0)
    torch.cuda.synchronize()
    for (t, s, e), buf in zip(boxes, bufs):
        ref = t[s[0]:s[0] + e[0], s[1]:s[1] + e[1], s[2]:s[2] + e[2]].permute(2, 1, 0).reshape(-1)
        assert torch.equal(buf, ref)
    a2, b2 = torch.zeros_like(a), torch.zeros_like(b)
    BatchedCopy([(t2, s, e, buf) for (t, s, e), buf, t2 in zip(boxes, bufs, (a2, a2, b2))]).run(1)
    torch.cuda.synchronize()
    for (t, s, e), t2 in zip(boxes, (a2, a2, b2)):
        sl = (slice(s[0], s[0] + e[0]), slice(s[1], s[1] + e[1]), slice(s[2], s[2] + e[2]))
        assert torch.equal(t2[sl], t[sl])


@pytest.mark.parametrize("dtype,ei,i0", [("float64", 2, 2), ("float64", 2, 3), ("float32", 4, 4),
                                          ("float32", 2, 1), ("float64", 3, 0), ("float64", 1, 5)])
def test_batched_halo_copy_narrow_faces(dtype, ei, i0):
    """I faces of the 2-D exchange (a few cells per row of an I-first field): the 16-B row path
    (aligned 16-B face rows) and the element path (other widths / alignments), pack and unpack."""
    torch = _torch()
    from gt4py_amd import storage
    from gt4py_amd.distributed.halo_copy import BatchedCopy

    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(ei * 10 + i0)
    t = storage.empty((40, 23, 5), np.dtype(dtype), backend=BACKEND, aligned_index=(0, 0, 0))
    t.copy_(torch.rand(t.shape, generator=g, device=dev, dtype=t.dtype))
    boxes = [(t, (i0, 0, 0), (ei, 23, 5)), (t, (40 - ei, 1, 1), (ei, 21, 4))]
    bufs = [torch.empty(e[0] * e[1] * e[2], dtype=t.dtype, device=dev) for _, _, e in boxes]
    BatchedCopy([(f, s, e, b) for (f, s, e), b in zip(boxes, bufs)]).run(0)
    torch.cuda.synchronize()
    for (f, s, e), b in zip(boxes, bufs):
        ref = f[s[0]:s[0] + e[0], s[1]:s[1] + e[1], s[2]:s[2] + e[2]].permute(2, 1, 0).reshape(-1)
        assert torch.equal(b, ref)
    t2 = storage.zeros((40, 23, 5), np.dtype(dtype), backend=BACKEND, aligned_index=(0, 0, 0))
    BatchedCopy([(t2, s, e, b) for (_, s, e), b in zip(boxes, bufs)]).run(1)
    torch.cuda.synchronize()
    for _, s, e in boxes:
        sl = (slice(s[0], s[0] + e[0]), slice(s[1], s[1] + e[1]), slice(s[2], s[2] + e[2]))
        assert torch.equal(t2[sl], t[sl])
    mask = torch.ones_like(t2, dtype=torch.bool)
    for _, s, e in boxes:
        mask[s[0]:s[0] + e[0], s[1]:s[1] + e[1], s[2]:s[2] + e[2]] = False
    assert float(t2[mask].abs().sum()) == 0.0  # nothing outside the boxes written
