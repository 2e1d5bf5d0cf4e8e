"""Layout maps (``src/gt4py/storage/cartesian/layout.py:21-76``).

A layout map gives, per dimension, its rank in memory order: the dimension with the
highest rank is contiguous. ``(2, 1, 0)`` = I contiguous, then J, then K ("I-first").
"""

from __future__ import annotations

from typing import Any, Callable, Literal, Sequence, Tuple, TypedDict

import numpy as np


class LayoutInfo(TypedDict):
    alignment: int  # in elements (multiplied by itemsize by the allocator, as in the reference)
    device: Literal["cpu", "gpu"]
    layout_map: Callable[[Tuple[str, ...]], Tuple[int, ...]]
    is_optimal_layout: Callable[[Any, Tuple[str, ...]], bool]


def layout_maker_factory(base_layout: Tuple[int, ...]) -> Callable[[Tuple[str, ...]], Tuple[int, ...]]:
    def layout_maker(dimensions: Tuple[str, ...]) -> Tuple[int, ...]:
        mask = [dim in dimensions for dim in "IJK"]
        ranks = [bl for m, bl in zip(mask, base_layout) if m]
        n_data = len(dimensions) - sum(mask)
        ranks = [n_data + r for r in ranks]
        ranks.extend(range(n_data))
        res = [0] * len(ranks)
        for i, idx in enumerate(np.argsort(ranks)):
            res[idx] = i
        return tuple(res)

    return layout_maker


def _strides_of(arr) -> Tuple[int, ...]:
    if isinstance(arr, np.ndarray):
        return tuple(arr.strides)
    st = arr.stride()
    item = arr.element_size()
    return tuple(s * item for s in st)


def check_layout(layout_map, strides) -> bool:
    if len(strides) != len(layout_map):
        return False
    stride = 0
    for dim in reversed(np.argsort(layout_map)):
        if strides[dim] < stride:
            return False
        stride = strides[dim]
    return True


def layout_checker_factory(layout_maker):
    def layout_checker(field, dimensions: Tuple[str, ...]) -> bool:
        return check_layout(layout_maker(dimensions), _strides_of(field))

    return layout_checker


def make_strides(shape: Sequence[int], layout_map: Sequence[int]) -> Tuple[int, ...]:
    """Element strides for ``shape`` laid out by ``layout_map`` (highest rank contiguous)."""
    ndim = len(shape)
    strides = [0] * ndim
    acc = 1
    for dim in sorted(range(ndim), key=lambda d: -layout_map[d]):
        strides[dim] = acc
        acc *= max(int(shape[dim]), 1)
    return tuple(strides)
