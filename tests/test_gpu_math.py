"""The device forms of the shared math (csrc/ngp_math.h) against the operations they replace, over whole input
ranges (ngp_debug_math_check). The sampler's and the loss pass's bit-exactness against the oracle rests on the
device and the host evaluating the same floats; where the device uses a shorter instruction sequence, this
checks that it gives the reference operation's result for every input it can receive."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_logf_division_equals_ieee_quotient_for_every_reduced_argument():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from __graft_entry__ import load_package
    lib = load_package().lib()
    bad = ctypes.c_uint64(123)
    assert lib.ngp_debug_math_check(0, None, ctypes.byref(bad)) == 0
    assert bad.value == 0  # all 2^23 values of f = m - 1, m in [sqrt(2)/2, sqrt(2))
    assert lib.ngp_debug_math_check(7, None, ctypes.byref(bad)) != 0  # unknown check: refused
