"""Full-frame helpers (utils.py:339-356, :464-537 restated in avr.video):
pixel grid, look-at rotation and the camera ring, checked on CPU against the
oracle's float64 restatement; the PPM writer round-trips."""
import numpy as np

from oracle import avr_oracle as O
from oracle import synth


def test_pixel_grid_matches_reference_quirk():
    from avr.video import get_opencv_pixel_coordinates
    for h, w in ((4, 4), (3, 5), (8, 6)):
        got = get_opencv_pixel_coordinates(h, w).numpy()
        np.testing.assert_array_equal(got.shape, (h, w, 2))
        np.testing.assert_allclose(got, O.opencv_pixel_coordinates(h, w), atol=1e-7)


def test_orbit_matches_generate_video_ring():
    import math
    from avr.video import orbit_cam2world
    n = 7
    poses = orbit_cam2world(n, 1.3)
    for i, c2w in enumerate(poses):
        angle = 2 * math.pi * i / n + math.pi / n      # linspace(0, 2 pi (n-1)/n, n) + pi/n
        np.testing.assert_allclose(c2w.numpy(), synth.orbit_cam2world(angle), atol=2e-6)


def test_get_R_is_a_rotation():
    from avr.video import get_R
    R = get_R(0.3, -1.1, 0.4)[0].numpy().astype(np.float64)
    np.testing.assert_allclose(R.T @ R, np.eye(3), atol=1e-6)
    np.testing.assert_allclose(np.linalg.det(R), 1.0, atol=1e-6)


def test_write_ppm(tmp_path):
    from avr.video import to_uint8, write_ppm
    img = np.random.default_rng(0).random((5, 3, 3)).astype(np.float32)
    f = to_uint8(img)
    p = tmp_path / "f.ppm"
    write_ppm(str(p), f)
    data = p.read_bytes()
    header = b"P6\n3 5\n255\n"
    assert data.startswith(header)
    np.testing.assert_array_equal(np.frombuffer(data[len(header):], np.uint8).reshape(5, 3, 3), f)
