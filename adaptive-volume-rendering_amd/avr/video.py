"""Full-frame rendering on the fused path: the reference's video utilities
(utils.py:339-356 get_opencv_pixel_coordinates, :464-479 get_R, :481-537
generate_video) with the same signatures and pose conventions, plus
`render_orbit`, a frame loop that takes a ready radiance field (no encoder)
and can terminate the fine pass early (BASELINE config 4).

Frames come back as uint8 (H, W, 3) numpy arrays like the reference's;
`write_ppm` stores them without an image library."""
import math
import time

import numpy as np
import torch
import torch.nn.functional as F


def get_opencv_pixel_coordinates(y_resolution, x_resolution):
    """utils.py:339-356. (y_res, x_res, 2) pixel coordinates in [0, 1), origin
    top-left; quirk Q8 kept: both axes step by 1 / x_resolution."""
    i, j = torch.meshgrid(torch.linspace(0, 1 - 1 / x_resolution, steps=x_resolution),
                          torch.linspace(0, 1 - 1 / x_resolution, steps=y_resolution), indexing="ij")
    return torch.stack([i.float(), j.float()], dim=-1).permute(1, 0, 2)


def get_R(x, y, z):
    """Look-at rotation of a camera at (x, y, z) aimed at the origin, with the
    scene's (0, 0, -1) reference direction (utils.py:464-479): (1, 3, 3) whose
    columns are the camera's x, y and viewing axes. When the viewing axis is
    (anti)parallel to the reference direction, x is rebuilt from y and the
    viewing axis, as the reference does."""
    eye = torch.tensor([[float(x), float(y), float(z)]], dtype=torch.float32)
    ref_dir = torch.tensor([[0.0, 0.0, -1.0]])
    view = F.normalize(torch.zeros(1, 3) - eye, eps=1e-5)
    cam_x = F.normalize(torch.cross(ref_dir, view, dim=1), eps=1e-5)
    cam_y = F.normalize(torch.cross(view, cam_x, dim=1), eps=1e-5)
    degenerate = torch.isclose(cam_x, torch.tensor(0.0), atol=5e-3).all(dim=1, keepdim=True)
    if bool(degenerate.any()):
        cam_x = torch.where(degenerate, F.normalize(torch.cross(cam_y, view, dim=1), eps=1e-5), cam_x)
    return torch.stack([cam_x, cam_y, view], dim=2)


def orbit_cam2world(num_frames, radius, z_height=0.4):
    """The camera ring of generate_video (utils.py:499-515): num_frames poses
    at height z_height on a circle of the given radius around the origin,
    OpenCV convention (x diag(1, -1, -1, 1)). Returns a list of (4, 4)."""
    angles = torch.linspace(0, 2 * np.pi * (num_frames - 1) / num_frames, num_frames) + np.pi / num_frames
    rradius = math.sqrt(radius * radius - z_height * z_height)
    flip = torch.diag(torch.tensor([1, -1, -1, 1], dtype=torch.float32))
    out = []
    for i in range(num_frames):
        angle = float(angles[i])
        tx, ty, tz = rradius * math.sin(angle), rradius * math.cos(angle), z_height
        c2w = torch.zeros(4, 4)
        c2w[:3, :3] = get_R(tx, ty, tz)[0]
        c2w[0, 3], c2w[1, 3], c2w[2, 3], c2w[3, 3] = tx, ty, tz, 1.0
        out.append(c2w @ flip)
    return out


def to_uint8(img):
    """The reference's frame conversion (utils.py:528-531)."""
    return np.clip(img * 255, 0, 255).astype(np.uint8)


def render_orbit(renderer, radiance_field, intrinsics, num_frames, radius, height, width=None, fine=True,
                 device=None, t_stop=None, on_frame=None):
    """Render num_frames full frames around the orbit with `renderer`
    (e.g. avr.renderers.VolumeRenderer) and a ready radiance field. One
    renderer call per frame (all H * W rays at once), no_grad. Returns
    (frames, stats): frames uint8 (H, W, 3); stats = seconds, rays/s and the
    fine samples evaluated (< H * W * (n_coarse + n_fine) once rays terminate)."""
    width = width or height
    device = device or intrinsics.device
    K = intrinsics.reshape(1, 3, 3).to(device)
    x_pix = get_opencv_pixel_coordinates(height, width).reshape(1, -1, 2).to(device)
    n = x_pix.shape[1]
    prev = getattr(renderer, "t_stop", None)
    renderer.t_stop = t_stop
    frames, fine_samples = [], 0
    try:
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        with torch.no_grad():
            for c2w in orbit_cam2world(num_frames, radius):
                c2w = c2w.to(device).reshape(1, 1, 4, 4).expand(1, n, 4, 4)
                rgb_c, rgb_f, _, _ = renderer(c2w, K, x_pix, radiance_field)
                fine_samples += getattr(renderer, "last_fine_samples", 0)
                img = (rgb_f if fine else rgb_c)[0].reshape(height, width, 3)
                frame = to_uint8(img.float().cpu().numpy())
                frames.append(frame)
                if on_frame is not None:
                    on_frame(len(frames) - 1, frame)
        torch.cuda.synchronize(device)
        secs = time.perf_counter() - t0
    finally:
        renderer.t_stop = prev
    return frames, {"seconds": secs, "rays_per_s": num_frames * n / secs, "frames": num_frames,
                    "rays_per_frame": n, "fine_samples": fine_samples}


def generate_video(model_input, num_frames, radius, net, model, fine=True):
    """utils.py:481-537 with the same arguments: encode the first source view
    of model_input into `net`, then render the orbit through `model`
    (a RadFieldAndRenderer). A net whose latent was set with encode_latent()
    keeps it (no `images` needed); otherwise the source view is encoded."""
    intrinsics = model_input["intrinsics"][0:1, 0, ...]
    if "images" in model_input and net.encoder.latent.shape[-1] <= 1:   # no latent yet
        gt = model_input["images"]
        _, _, sl2, _ = gt.shape
        sl = int(np.sqrt(sl2))
        src = gt[0:1, 0:1, ...].reshape(1, -1, sl, sl, 3).permute(0, 1, 4, 2, 3)
        net.encode(src, model_input["cam2world"][0:1, 0:1, ...], model_input["focal"][0, 0], model_input["c"][0, 0, :])
    sl = int(model_input.get("resolution", 0)) or int(np.sqrt(model_input["images"].shape[2]))
    frames, stats = render_orbit(model.renderer, net, intrinsics, num_frames, radius, sl, fine=fine)
    print(f"it takes {stats['seconds']} seconds to render a video")
    return frames


def write_ppm(path, frame):
    """Binary PPM (P6) of a uint8 (H, W, 3) frame."""
    h, w, _ = frame.shape
    with open(path, "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (w, h))
        f.write(np.ascontiguousarray(frame, dtype=np.uint8).tobytes())
