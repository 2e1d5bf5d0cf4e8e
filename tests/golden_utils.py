"""Loader for the golden fixtures produced by tests/golden/make_golden.py."""

import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def available():
    return sorted(f[:-4] for f in os.listdir(GOLDEN_DIR) if f.endswith(".npz"))


def load(name):
    with np.load(os.path.join(GOLDEN_DIR, f"{name}.npz"), allow_pickle=False) as z:
        inputs, outputs = {}, {}
        for key in z.files:
            if key.startswith("in__"):
                inputs[key[4:]] = z[key]
            elif key.startswith("out__"):
                outputs[key[5:]] = z[key]
        meta = json.loads(bytes(z["meta_json"]).decode())
    return inputs, outputs, meta


def assert_match(actual, expected, rtol=0.0, atol=0.0, name=""):
    actual = np.asarray(actual)
    expected = np.asarray(expected)
    assert actual.shape == expected.shape, (name, actual.shape, expected.shape)
    assert actual.dtype == expected.dtype, (name, actual.dtype, expected.dtype)
    if rtol == 0.0 and atol == 0.0:
        if actual.dtype.kind == "f":
            same = (actual == expected) | (np.isnan(actual) & np.isnan(expected))
            if not same.all():
                bad = np.argwhere(~same)
                idx = tuple(bad[0])
                raise AssertionError(
                    f"{name}: {len(bad)} mismatches (bit-exact expected); first at {idx}: "
                    f"{actual[idx]!r} != {expected[idx]!r}"
                )
        else:
            np.testing.assert_array_equal(actual, expected, err_msg=name)
    else:
        np.testing.assert_allclose(actual, expected, rtol=rtol, atol=atol, equal_nan=True, err_msg=name)
