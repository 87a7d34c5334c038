"""Dataset-side ray batching of one train.py step (train.py:53-83, utils.py:34-60):
choose each scene's source view, sample the ray batch (uniformly, or inside
each view's object bounding box) and gather the per-ray inputs the renderer
takes, with the reference's draw order (torch.randint source index, then ray
indices; bbox_sample: randint view, rand x, rand y). The draws come from the
CPU generator by default, as in train.py (its torch.randint / bbox_sample calls
run on the collated CPU batch), so a batch that already lives on the GPU gets
the same indices as the reference; the gathers run on the batch's device.

Loading the HDF5 scenes (dataset.py, h5py + torchvision transforms) is host
I/O outside this package; `all_input` is the collated dict it produces:
images (SB, NV, H*W, 3) in [-1, 1], cam2world (SB, NV, 4, 4), intrinsics
(SB, NV, 3, 3), focal (SB, NV), c (SB, NV, 2), x_pix (SB, NV, H*W, 2),
bbox (SB, NV, 4) = [cmin, rmin, cmax, rmax].
"""
import math

import torch


def batched_index_select_nd(t, inds):
    """utils.py:34-43: index select on dim 1 of (batch, n, ...) with (batch, k)."""
    return t.gather(1, inds[(...,) + (None,) * (len(t.shape) - 2)].expand(-1, -1, *t.shape[2:]))


def bbox_sample(bboxes, num_pix, generator=None):
    """utils.py:45-60: num_pix pixels inside random views' boxes -> (num_pix, 3) = (view, y, x)."""
    dev = bboxes.device
    image_ids = torch.randint(0, bboxes.shape[0], (num_pix,), generator=generator, device=dev)
    b = bboxes[image_ids]
    x = (torch.rand(num_pix, generator=generator, device=dev) * (b[:, 2] + 1 - b[:, 0]) + b[:, 0]).long()
    y = (torch.rand(num_pix, generator=generator, device=dev) * (b[:, 3] + 1 - b[:, 1]) + b[:, 1]).long()
    return torch.stack((image_ids, y, x), dim=-1)


def sample_ray_batch(all_input, ray_batch_size, with_bbox=False, num_source=1, generator=None, draw_device="cpu"):
    """One step's inputs (train.py:53-83) -> (source, model_input, ground_truth):
      source       dict(images (SB, NS, 3, sl, sl), poses (SB, NS, 4, 4), focal (), c (2,)) for net.encode
      model_input  dict(x_pix (SB, R, 2), cam2world (SB, R, 4, 4), intrinsics (SB, 3, 3)) for the renderer
      ground_truth (SB, R, 3) in [0, 1].
    draw_device: where the random indices are drawn ("cpu": the reference's generator and results whatever
    device the batch is on; None: the batch's device)."""
    images = all_input["images"]
    SB, NV, sl2, _ = images.shape
    dev = images.device
    ddev = dev if draw_device is None else torch.device(draw_device)
    sl = int(math.isqrt(sl2))
    NS = num_source
    src_idx = torch.randint(0, NV, (SB, NS), generator=generator, device=ddev).to(dev)
    src_images = batched_index_select_nd(images, src_idx).reshape(SB, NS, sl, sl, 3).permute(0, 1, 4, 2, 3)
    source = {"images": src_images,
              "poses": batched_index_select_nd(all_input["cam2world"], src_idx),
              "focal": batched_index_select_nd(all_input["focal"], src_idx)[0, 0],
              "c": batched_index_select_nd(all_input["c"], src_idx)[0, 0, :]}
    if with_bbox:
        rays_idx = []
        for sb in range(SB):
            pix = bbox_sample(all_input["bbox"][sb].to(ddev), ray_batch_size, generator)
            rays_idx.append(pix[..., 0] * sl2 + pix[..., 1] * sl + pix[..., 2])
        rays_idx = torch.stack(rays_idx).to(dev)
    else:
        rays_idx = torch.randint(0, NV * sl2, (SB, ray_batch_size), generator=generator, device=ddev).to(dev)
    c2w = all_input["cam2world"].unsqueeze(2).expand(SB, NV, sl2, 4, 4).reshape(SB, -1, 4, 4)
    model_input = {"x_pix": batched_index_select_nd(all_input["x_pix"].reshape(SB, -1, 2), rays_idx),
                   "cam2world": batched_index_select_nd(c2w, rays_idx),
                   "intrinsics": all_input["intrinsics"][:, 0, ...]}
    ground_truth = 0.5 * batched_index_select_nd(images.reshape(SB, -1, 3), rays_idx) + 0.5
    return source, model_input, ground_truth
