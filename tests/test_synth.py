"""The synthetic corridor generator."""
import numpy as np


def test_deterministic_and_shaped(synth):
    a = synth.make_scan(3)
    b = synth.make_scan(3)
    assert a.shape == (64, 1024, 4) and a.dtype == np.float32
    assert np.array_equal(a, b)
    assert not np.array_equal(a, synth.make_scan(4))


def test_dropouts_and_intensity_clamp(synth):
    a = synth.make_scan(0)
    zero = np.all(a == 0, axis=-1)
    assert 0.01 < zero.mean() < 0.03
    assert (a[..., 3] > 255).any() and (a[..., 3] <= 300).all()


def test_beams_at_scanid_bin_centres(synth):
    import restate_np as R

    for H in (16, 32, 64, 128):
        el = synth.beam_elevations_deg(H).astype(np.float32)
        assert np.array_equal(R.scan_id(el, H), np.arange(H))
        for d in (-0.2, 0.2):  # robust to perturbations far beyond 1 ulp
            assert np.array_equal(R.scan_id((el + np.float32(d / (1.41 if H == 64 else 2.83 if H == 128 else 3.0)))
                                            .astype(np.float32), H), np.arange(H))
