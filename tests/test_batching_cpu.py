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


def test_train_py_encode_call_uses_image_centre(golden):
    """train.py:68 calls net.encode(src_images, poses, focal, c): c lands in the
    4th positional slot, z_bounds, which the reference ignores (models.py:682-733),
    so the principal point is the image centre whatever source['c'] holds.
    The same call on avr.models.NewPixelNeRFNet behaves the same way."""
    from avr.batching import sample_ray_batch
    from avr.models import NewPixelNeRFNet
    from helpers import model_conf
    g = golden("g8_batching.npz")
    all_input = {k: torch.from_numpy(g[k]) for k in ("images", "cam2world", "intrinsics", "focal", "c", "x_pix",
                                                     "bbox")}
    torch.manual_seed(int(g["bbox0_seed"]))
    src, _, _ = sample_ray_batch(all_input, 16)
    conf = model_conf(64, 3, 1000, 64)
    conf["encoder"] = {"backbone": "resnet34", "pretrained": False, "num_layers": 1}
    net = NewPixelNeRFNet(conf).eval()
    with torch.no_grad():
        net.encode(src["images"], src["poses"], src["focal"], src["c"])     # train.py:68, positional
    sl = src["images"].shape[-1]
    np.testing.assert_array_equal(net.c.numpy(), [[sl * 0.5, sl * 0.5]])
    assert not np.allclose(src["c"].numpy(), sl * 0.5)   # the dataset's c really is dropped, not equal by chance
