"""The fp32 kernels' branch-free GELU (cdna4_common.h gelu_erfc_nr: x·Φ(x) with the Chebyshev
erfc of Numerical Recipes) against float64 erf: |Δ| <= 2e-7·max(1, |x|) in float32 emulation."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import gelu_error  # noqa: E402


def test_gelu_erfc_nr_error_bound():
    assert gelu_error.max_error() <= 2e-7


def test_gelu_as_f32_error_bound():
    """gelu_as_f32 (Abramowitz & Stegun 7.1.26) in the device's operation order: <= 2.5e-7·max(1, |x|)."""
    assert gelu_error.max_error(gelu_error.gelu_as) <= 2.5e-7


def test_gelu_as_f32x2_error_bound():
    """gelu_as_f32x2 (the packed-fp32 form, constants folded): the same <= 2.5e-7·max(1, |x|)."""
    assert gelu_error.max_error(gelu_error.gelu_as_pk) <= 2.5e-7
