"""Dataset-side ray batching (train.py:53-83) against the reference's own
utils.batched_index_select_nd / bbox_sample run with the same seeds
(tests/golden/g8_batching.npz, make_golden.py)."""
import numpy as np
import pytest
import torch


@pytest.mark.parametrize("with_bbox", [False, True])
def test_sample_ray_batch_matches_reference(golden, with_bbox):
    from avr.batching import sample_ray_batch
    g = golden("g8_batching.npz")
    all_input = {k: torch.from_numpy(g[k]) for k in ("images", "cam2world", "intrinsics", "focal", "c", "x_pix",
                                                     "bbox")}
    k = f"bbox{int(with_bbox)}"
    torch.manual_seed(int(g[f"{k}_seed"]))
    src, mi, gt = sample_ray_batch(all_input, 16, with_bbox=with_bbox)
    np.testing.assert_array_equal(src["images"].numpy(), g[f"{k}_src_images"])
    np.testing.assert_array_equal(src["poses"].numpy(), g[f"{k}_poses"])
    np.testing.assert_array_equal(src["focal"].numpy(), g[f"{k}_focal"])
    np.testing.assert_array_equal(src["c"].numpy(), g[f"{k}_c"])
    np.testing.assert_array_equal(mi["x_pix"].numpy(), g[f"{k}_x_pix"])
    np.testing.assert_array_equal(mi["cam2world"].numpy(), g[f"{k}_cam2world"])
    np.testing.assert_array_equal(gt.numpy(), g[f"{k}_gt"])
    np.testing.assert_array_equal(mi["intrinsics"].numpy(), g["intrinsics"][:, 0])


def test_bbox_sample_inside_boxes():
    from avr.batching import bbox_sample
    gen = torch.Generator().manual_seed(0)
    boxes = torch.tensor([[1.0, 2.0, 5.0, 6.0], [0.0, 0.0, 0.0, 0.0]])
    pix = bbox_sample(boxes, 4000, gen)
    b = boxes[pix[:, 0]]
    assert bool(((pix[:, 2] >= b[:, 0]) & (pix[:, 2] <= b[:, 2]) & (pix[:, 1] >= b[:, 1]) & (pix[:, 1] <= b[:, 3])).all())
