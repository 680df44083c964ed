"""The GPU elimination's retry rule on the CPU (tests/panel_rule.py, a model
of gf_elim.hip's attempts): the row rotation and its undoing give C^-1, the
attempts reach every invertible C the first one misses, and the abort rules
(a singular C, a structured batch) never give up on an invertible random C.
No GPU: the GPU side is tests/test_gpu_elim_route.py."""
import numpy as np
import pytest

import panel_rule as pr


@pytest.mark.parametrize("k", [32, 48, 64, 100])
def test_rotation_undone_gives_the_inverse(k):
    rng = np.random.default_rng(k)
    C = rng.integers(0, 256, (k, k), dtype=np.uint8)
    T = pr.gf_inverse(C)
    assert T is not None
    for a in range(pr.ATTEMPTS):
        s = pr.rot(a, k)
        Tp = pr.gf_inverse(pr.rotate_rows(C, s))
        assert np.array_equal(pr.unrotate_columns(Tp, s), T)


@pytest.mark.parametrize("seed", [7, 8])
def test_singular_panel_seeds_succeed_on_a_later_attempt(seed):
    """profiles/r04/c2_seeds/: the device vectors of seeds 7 and 8 (k = 256)
    fail the first attempt (a singular leading panel block) though C is
    invertible; a rotated attempt succeeds."""
    C = pr.device_vectors(seed, 256, 256)
    assert pr.attempt(C) == "retry"
    a = pr.expected_attempt(C)
    assert a is not None and a >= 1
    assert pr.gf_inverse(C) is not None


def test_random_invertible_batches_never_fall_back():
    rng = np.random.default_rng(5)
    k, n, retried = 48, 400, 0
    for _ in range(n):
        C = rng.integers(0, 256, (k, k), dtype=np.uint8)
        a = pr.expected_attempt(C)
        inv_ok = pr.gf_inverse(C) is not None
        if a is None:
            # only a singular C (or, at 6 %^4 odds, four failed orders) leaves the GPU
            assert not inv_ok
        else:
            assert inv_ok
            retried += a > 0
    assert retried > 0  # the first order fails ~k/16/255 of the time: some retried


def test_singular_and_structured_batches_abort_at_once():
    rng = np.random.default_rng(9)
    k = 64
    C = rng.integers(0, 256, (k, k), dtype=np.uint8)
    C[k - 1] = C[3] ^ pr.mul(7, C[10]).astype(np.uint8)  # a dependent last row: C singular
    assert pr.attempt(C) == "abort"
    assert pr.expected_attempt(C) is None
    # systematic order with a loss: a panel block with a zero column
    eye = np.eye(k, dtype=np.uint8)[[i for i in range(k) if i != 5]]
    S = np.concatenate([eye, rng.integers(0, 256, (1, k), dtype=np.uint8)])
    assert pr.attempt(S) == "abort"
