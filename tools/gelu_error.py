"""Error of the fp32 GELU of the parity kernels (cdna4_common.h gelu_erfc_nr) against float64,
emulated in float32 numpy (the device's v_rcp_f32 / v_exp_f32 add about 1 ulp each).

    python tools/gelu_error.py      -> max |Δ| / max(1, |x|) over [-10, 10] and log grids
"""
from math import erfc, sqrt

import numpy as np

f32 = np.float32
C = [0.17087277, -0.82215223, 1.48851587, -1.13520398, 0.27886807, -0.18628806, 0.09678418, 0.37409196,
     1.00002368, -1.26551223]


def gelu_nr(x):
    x = f32(x)
    z = f32(abs(x) * f32(0.70710678118654752440))
    t = f32(1) / f32(f32(1) + f32(0.5) * z)
    q = f32(C[0])
    for k in C[1:]:
        q = f32(f32(q * t) + f32(k))
    y = f32(f32(-z * z) + q)
    ec = f32(t * f32(np.exp2(f32(y * f32(1.4426950408889634)))))
    phi = f32(0.5) * ec if x < 0 else f32(1) - f32(0.5) * ec
    return f32(x * phi)


def gelu_as(x):
    """cdna4_common.h gelu_as_f32 (Abramowitz & Stegun 7.1.26 erf) in the device's operation order."""
    x = f32(x)
    z = f32(abs(x) * f32(0.70710678118654752440))
    t = f32(1) / f32(f32(f32(0.3275911) * z) + f32(1))
    q = f32(f32(f32(1.061405429) * t) + f32(-1.453152027))
    for k in (1.421413741, -0.284496736, 0.254829592):
        q = f32(f32(q * t) + f32(k))
    q = f32(q * t)
    e = f32(np.exp2(f32(f32(-1.4426950408889634) * f32(z * z))))
    erfz = f32(f32(1) - f32(q * e))
    hx = f32(f32(0.5) * x)
    return f32(f32(hx * f32(np.copysign(erfz, x))) + hx)


def gelu_as_pk(x):
    """cdna4_common.h gelu_as_f32x2 (the packed-fp32 form of gelu_as_f32): the 1/sqrt(2) folded into
    the denominator's coefficient and the exponent's, the rest in the same order."""
    x = f32(x)
    t = f32(1) / f32(f32(f32(f32(0.3275911) * f32(0.70710678118654752440)) * f32(abs(x))) + f32(1))
    q = f32(f32(f32(1.061405429) * t) + f32(-1.453152027))
    for k in (1.421413741, -0.284496736, 0.254829592):
        q = f32(f32(q * t) + f32(k))
    q = f32(q * t)
    e = f32(np.exp2(f32(f32(x * x) * f32(-0.72134752044448170368))))
    erfz = f32(f32(1) - f32(q * e))
    hx = f32(x * f32(0.5))
    return f32(f32(hx * f32(np.copysign(erfz, x))) + hx)


def max_error(fn=gelu_nr):
    xs = np.concatenate([np.linspace(-10, 10, 200001), np.logspace(-8, 1, 2000), -np.logspace(-8, 1, 2000)])
    worst = 0.0
    for x in xs:
        ref = 0.5 * x * erfc(-x / sqrt(2))
        worst = max(worst, abs(float(fn(x)) - ref) / max(1.0, abs(x)))
    return worst


if __name__ == "__main__":
    print(f"max |gelu_nr - gelu| / max(1, |x|) = {max_error(gelu_nr):.3e}")
    print(f"max |gelu_as - gelu| / max(1, |x|) = {max_error(gelu_as):.3e}")
    print(f"max |gelu_as_pk - gelu| / max(1, |x|) = {max_error(gelu_as_pk):.3e}")
