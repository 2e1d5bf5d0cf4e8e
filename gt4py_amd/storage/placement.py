"""HBM placement tuning for the fields a stencil writes (DESIGN.md §5 "HBM placement").

On MI355X the time of a bandwidth-bound stencil depends, for one and the same library and
inputs, on the physical HBM pages its WRITTEN fields occupy: hdiff 2048x2048x160 f64 measures
2.50, 2.63 or 2.80 ms depending only on where ``out_field`` lives, reproducibly per buffer
(+-0.3 %), with a box-specific pattern (``scripts/placement_scan.py``,
``profiles/r03/r03b_placement_scan.jsonl``). The physical address is private to the kernel
driver, so no address rule can pick a good buffer; a measurement can. The fields of a simulation
are allocated once and stepped thousands of times, so measuring a few buffers once pays back:

    arrays, report = tune_written_fields(stencil, {"in_field": a, "out_field": b, "coeff": c},
                                         origin=..., domain=..., candidates=3)

keeps every read-only field as it is, gives each written field ``candidates`` other buffers of
the same layout (same strides, same address residue modulo 2 MiB, so alignment and the HBM
stagger of :mod:`gt4py_amd.storage` are preserved), times the call on each set (HIP events,
median of ``reps`` launches on torch's current stream) and returns the arrays with the written
fields in the fastest set, holding the contents they had before (restored from a copy: the
timing launches write them; the caller's original arrays are restored too, also when a call
raises). The report lists every set's time; the unchosen buffers are freed.

Drop-in form: ``stencil.tune_placement(*args, origin=..., domain=..., candidates=3, **params)`` (and
``FrozenStencil.tune_placement(**kwargs)``) takes the arguments of an ordinary call and re-homes
the written fields IN PLACE (:func:`tune_in_place`): the caller's tensor objects stay the same and
now live on the chosen buffers, so a reference-API user opts in with one line and re-plumbs
nothing.

The reference has no counterpart: its storages are plain CuPy/NumPy allocations
(``/root/reference/src/gt4py/storage/cartesian/interface.py:143-327``); this tool only returns
other allocations of the same layout, so everything downstream sees ordinary fields.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

from gt4py_amd.definitions import AccessKind

_RESIDUE = 2 << 20  # keep the address residue modulo 2 MiB (the stagger quantum pair)


def like(t):
    """A new device tensor with ``t``'s sizes and strides whose first element has the same address
    residue modulo 2 MiB (alignment of the compute origin and the HBM stagger are kept)."""
    import torch

    span = 1 + sum((s - 1) * st for s, st in zip(t.shape, t.stride())) if t.numel() else 0
    item = t.element_size()
    buf = torch.empty(span + _RESIDUE // item, dtype=t.dtype, device=t.device)
    off = ((t.data_ptr() - buf.data_ptr()) % _RESIDUE) // item
    return torch.as_strided(buf, size=tuple(t.shape), stride=tuple(t.stride()), storage_offset=int(off))


def written_fields(stencil) -> List[str]:
    """Names of the API fields the stencil writes (``field_info`` access has WRITE)."""
    return [n for n, fi in stencil.field_info.items() if fi is not None and fi.access & AccessKind.WRITE]


def scope_fields(stencil, scope: str) -> List[str]:
    """The fields a tuning run re-homes: ``"written"`` (the default; what decides a plane
    kernel's placement mode) or ``"all"`` API fields the stencil accesses (a column kernel at one
    wave per SIMD is latency-bound on every stream it reads: vadv, 1 written field of 5, stays
    ~12 % slow on a fresh process's first allocation however its written field is placed;
    DESIGN.md §5 "the column kernels have placement modes too")."""
    if scope == "written":
        return written_fields(stencil)
    if scope == "all":
        return [n for n, fi in stencil.field_info.items() if fi is not None]
    raise ValueError(f"placement scope must be 'written' or 'all', got {scope!r}")


def _time_call(call, reps: int) -> float:
    import torch

    call()  # warm (first launch on new buffers: page-table walks)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record()
        call()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in evs)
    return float(t[len(t) // 2])


def tune_written_fields(
    stencil,
    arrays: Dict[str, Any],
    *,
    origin=None,
    domain=None,
    params: Optional[Dict[str, Any]] = None,
    candidates: int = 3,
    reps: int = 10,
    memory_fraction: float = 0.8,
) -> Tuple[Dict[str, Any], Dict[str, Any]]:
    """Place the written fields of ``stencil(**arrays, **params, origin=origin, domain=domain)``
    in the fastest of ``candidates + 1`` buffer sets (set 0 = the given arrays).

    Returns ``(arrays, report)``: ``arrays`` maps every name to the field to use from now on (the
    read-only ones unchanged), ``report`` = ``{"written", "fields", "candidates_ms", "chosen",
    "untuned_ms", "tuned_ms"}``. Written fields keep their contents. Raises ``ValueError`` if a written field
    shares memory with another argument (re-homing it would break the aliasing) and ``TypeError``
    for non-device arrays; fewer sets are tried when free device memory is short.
    """
    return tune_fields(stencil, arrays, written_fields(stencil), origin=origin, domain=domain, params=params,
                       candidates=candidates, reps=reps, memory_fraction=memory_fraction)


def tune_fields(
    stencil,
    arrays: Dict[str, Any],
    names: List[str],
    *,
    origin=None,
    domain=None,
    params: Optional[Dict[str, Any]] = None,
    candidates: int = 3,
    reps: int = 10,
    memory_fraction: float = 0.8,
) -> Tuple[Dict[str, Any], Dict[str, Any]]:
    """:func:`tune_written_fields` for an explicit list of field ``names`` (read-only fields may be
    among them: they are copied into each candidate set the same way)."""
    import torch

    params = dict(params or {})
    names = list(names)
    missing = [n for n in names if n not in arrays]
    if missing:
        raise ValueError(f"tune_written_fields: field(s) {missing} not among the arrays")
    for n in names:
        t = arrays[n]
        if not (isinstance(t, torch.Tensor) and t.is_cuda):
            raise TypeError(f"tune_written_fields: '{n}' is not a device tensor")
        for m, u in arrays.items():
            if m != n and isinstance(u, torch.Tensor) and u.is_cuda and \
                    u.untyped_storage().data_ptr() == t.untyped_storage().data_ptr():
                raise ValueError(f"tune_written_fields: field '{n}' shares memory with '{m}'")
    report: Dict[str, Any] = {"written": [n for n in written_fields(stencil) if n in names], "fields": names,
                              "candidates_ms": [], "chosen": 0}

    def call_with(sub):
        a = dict(arrays)
        a.update(sub)
        return lambda: stencil(**a, **params, origin=origin, domain=domain, validate_args=False)

    if not names:  # nothing written: nothing to place (and the call changes no field)
        stencil(**arrays, **params, origin=origin, domain=domain)  # full argument checks once
        report["candidates_ms"] = [_time_call(call_with({}), reps)]
        report["untuned_ms"] = report["tuned_ms"] = report["candidates_ms"][0]
        return dict(arrays), report

    per_set = sum(like_bytes(arrays[n]) for n in names)
    free, _ = torch.cuda.mem_get_info(arrays[names[0]].device)
    # the backup copy plus the candidate sets must fit in a fraction of what is free
    fit = int(free * memory_fraction // max(per_set, 1)) - 1
    n_sets = max(0, min(int(candidates), fit))
    report["sets_tried"] = n_sets + 1
    backup = {n: arrays[n].clone() for n in names}
    sets: List[Dict[str, Any]] = [{n: arrays[n] for n in names}]
    for _ in range(n_sets):  # all alive at once: each set lands on pages of its own
        sets.append({n: like(arrays[n]) for n in names})
    for s in sets[1:]:
        for n in names:
            s[n].copy_(backup[n])
    try:
        # full argument checks once (shapes, origins, domain against the fields' extents): the
        # timed launches skip validation, as a cached call does
        stencil(**arrays, **params, origin=origin, domain=domain)
        times = [_time_call(call_with(s), reps) for s in sets]
    finally:
        for n in names:  # the caller's own arrays keep their contents whatever happens
            arrays[n].copy_(backup[n])
    best = min(range(len(times)), key=times.__getitem__)
    chosen = sets[best]
    for n in names:
        chosen[n].copy_(backup[n])
    out = dict(arrays)
    out.update(chosen)
    del backup, sets
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    report.update(candidates_ms=[round(t, 4) for t in times], chosen=best,
                  untuned_ms=round(times[0], 4), tuned_ms=round(times[best], 4))
    return out, report


def like_bytes(t) -> int:
    """Bytes a :func:`like` copy of ``t`` allocates."""
    span = 1 + sum((s - 1) * st for s, st in zip(t.shape, t.stride())) if t.numel() else 0
    return span * t.element_size() + _RESIDUE


def _storage_refs(t) -> Optional[int]:
    use = getattr(__import__("torch")._C, "_storage_Use_Count", None)
    if use is None:
        return None
    st = t.untyped_storage()
    return int(use(st._cdata)) - 1  # minus the temporary storage object itself


def _exclusive(t) -> bool:
    """``t`` is the only tensor on its storage (besides the flat buffer a gt4py_amd storage is a
    strided view of): re-homing it cannot leave another view writing the old pages."""
    import sys

    refs = _storage_refs(t)
    if refs is None:  # no use count in this torch: accept only tensors that are not views
        return t._base is None
    if t._base is None:
        return refs <= 1
    # a view: only of a flat buffer nothing else holds (getrefcount: the view's own reference
    # plus the call's argument)
    return refs <= 2 and t._base._base is None and sys.getrefcount(t._base) <= 2


def tune_in_place(
    stencil,
    arrays: Dict[str, Any],
    *,
    origin=None,
    domain=None,
    params: Optional[Dict[str, Any]] = None,
    candidates: int = 3,
    reps: int = 10,
    memory_fraction: float = 0.8,
    scope: str = "written",
) -> Dict[str, Any]:
    """:func:`tune_written_fields` (``scope="all"``: :func:`tune_fields` over every API field,
    :func:`scope_fields`), then move each field the tuner re-homed into the CALLER'S tensor object (``torch.utils.swap_tensors``): same object, same sizes, strides,
    dtype and contents, new buffer; the old buffer is freed. Returns the report (with
    ``"in_place": True``).

    Raises ``ValueError`` (before anything is timed) for a written field that other tensors view
    (they would keep the old pages) and ``RuntimeError`` (also before timing) if a field is weakly
    referenced outside gt4py_amd; gt4py_amd's own prepared launches and packed-argument caches are dropped first
    (they hold weak references and borrowed pointers; the next call re-prepares them).
    """
    import torch

    names = scope_fields(stencil, scope)
    for n in names:
        t = arrays.get(n)
        if not (type(t) is torch.Tensor and t.is_cuda):
            raise TypeError(f"tune_placement: '{n}' is not a plain device torch.Tensor")
        if not _exclusive(t):
            raise ValueError(f"tune_placement: field '{n}' shares its storage with other tensors "
                             f"(views would keep the old buffer); use tune_written_fields and pass the returned arrays")
    # weak references held outside gt4py_amd: refused before anything is timed (our own prepared
    # launches and packed-argument caches are dropped first; they re-prepare on the next call)
    import weakref

    from gt4py_amd.stencil_object import drop_prepared_launches

    drop_prepared_launches()
    held = [n for n in names if weakref.getweakrefcount(arrays[n])]
    if held:
        raise RuntimeError(f"tune_placement: field(s) {held} are weakly referenced elsewhere; cannot re-home "
                           "them in place (use tune_written_fields)")
    out, report = tune_fields(stencil, arrays, names, origin=origin, domain=domain, params=params,
                              candidates=candidates, reps=reps, memory_fraction=memory_fraction)
    report["scope"] = scope
    moved = [n for n in names if out[n] is not arrays[n]]
    if moved:
        drop_prepared_launches()  # the tuner's own timing calls prepared launches again
        held = [n for n in moved if weakref.getweakrefcount(arrays[n])]
        if held:
            raise RuntimeError(f"tune_placement: field(s) {held} are weakly referenced elsewhere; cannot re-home "
                               "them in place (use tune_written_fields)")
        for n in moved:
            torch.utils.swap_tensors(arrays[n], out[n])  # arrays[n] now holds the chosen buffer
        del out
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    report["in_place"] = True
    return report
