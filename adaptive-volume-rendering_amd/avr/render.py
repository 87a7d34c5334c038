"""Full-frame render CLI (the reference's generate_video
harness, utils.py:481-537, on the fused path; BASELINE configs 4 and 5).

    python -m avr.render --frames 4 --res 800 [--t-stop 1e-5] [--out DIR]
    torchrun --nproc-per-node N -m avr.render ...   # rays of every frame sharded over N GPUs

Renders `--frames` views on the reference's camera ring (radius, height 0.4)
of the synthetic scene (avr.scene) or of a NewPixelNeRFNet state_dict
(`--weights`, loaded with weights_only=True) and a latent map (`--latent`,
.npy (1, 512, H, W)). Prints one JSON line with rays/s and the fine samples
evaluated; `--out` writes PPM frames. Multi-GPU: every rank renders its
64-ray tiles of each frame and one RCCL all_gather assembles the frame
(avr.parallel.render_sharded); the scene (weights, latent, source view) is
broadcast from rank 0 once before the first frame (avr.parallel.broadcast_scene)."""
import argparse
import json
import os
import time

import numpy as np
import torch


def build_net(args, device):
    from .scene import synthetic_scene
    net = synthetic_scene(device, args.seed, sigma_bias=args.sigma_bias)
    if args.weights:
        sd = torch.load(args.weights, map_location=device, weights_only=True)
        missing, unexpected = net.load_state_dict(sd, strict=False)
        bad = [k for k in missing if not k.startswith("encoder.")]
        if bad or unexpected:
            raise SystemExit(f"--weights: missing {bad[:5]} unexpected {list(unexpected)[:5]}")
    if args.latent:
        lat = torch.from_numpy(np.load(args.latent, allow_pickle=False)).float().to(device)
        net.encoder.set_latent(lat)
    net.field_precision = args.precision
    return net


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--res", type=int, default=800, help="frame height = width (rays per frame = res^2)")
    ap.add_argument("--radius", type=float, default=1.3)
    ap.add_argument("--n-coarse", type=int, default=128)
    ap.add_argument("--n-fine", type=int, default=64)
    ap.add_argument("--near", type=float, default=0.8)
    ap.add_argument("--far", type=float, default=1.8)
    ap.add_argument("--t-stop", type=float, default=None, help="early ray termination of the fine pass")
    ap.add_argument("--precision", choices=["x3", "fp32"], default="x3")
    ap.add_argument("--sigma-bias", type=float, default=0.0, help="synthetic scene: density bias (opacity)")
    ap.add_argument("--weights", default=None, help="NewPixelNeRFNet state_dict (torch.save)")
    ap.add_argument("--latent", default=None, help=".npy latent map (1, 512, H, W)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--warmup", type=int, default=1, help="untimed frames first")
    ap.add_argument("--renderer", choices=["volume", "adaptive"], default="volume",
                    help="VolumeRenderer (coarse/fine) or AdaptiveVolumeRenderer (LSTM march + band)")
    ap.add_argument("--raymarch-steps", type=int, default=10)
    ap.add_argument("--epsilon", type=float, default=0.05)
    ap.add_argument("--out", default=None, help="directory for frame_XXX.ppm")
    args = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)

    from . import load_library
    from .parallel import render_sharded
    from .renderers import AdaptiveVolumeRenderer, VolumeRenderer
    from .scene import INTRINSICS
    from .video import get_opencv_pixel_coordinates, orbit_cam2world, to_uint8, write_ppm
    load_library()
    net = build_net(args, device)
    if dist is not None:
        # every rank renders rank 0's scene: weights, latent map and source view from rank 0 (one collective per
        # dtype; the receivers' packed-weight / table caches are invalidated)
        from .parallel import broadcast_scene
        broadcast_scene(net, src=0)
    if args.renderer == "adaptive":
        torch.manual_seed(args.seed + 2)
        rend = AdaptiveVolumeRenderer(net.d_latent, args.raymarch_steps, args.epsilon, args.n_coarse, True).to(device)
        samples_per_ray = args.n_coarse + 1 + args.raymarch_steps   # band + coarse point (+ LSTM lookups)
    else:
        rend = VolumeRenderer(args.near, args.far, args.n_coarse, args.n_fine, 0, 0.01, True)
        rend.seed = 1234
        rend.t_stop = args.t_stop
        samples_per_ray = args.n_coarse + args.n_fine
    K = torch.tensor([INTRINSICS], device=device)
    H = W = args.res
    x_pix = get_opencv_pixel_coordinates(H, W).reshape(1, -1, 2).to(device)
    n = x_pix.shape[1]
    poses = orbit_cam2world(args.frames, args.radius)

    def render(c2w):
        c2w = c2w.to(device).reshape(1, 1, 4, 4).expand(1, n, 4, 4)
        with torch.no_grad():
            if dist is None:
                return rend(c2w, K, x_pix, net)
            if isinstance(rend, VolumeRenderer):   # Philox keyed by frame-wide ray ids
                return render_sharded(lambda c, k, x, **ids: rend(c, k, x, net, **ids), c2w, K, x_pix,
                                      pass_ray_ids=True)
            return render_sharded(lambda c, k, x: rend(c, k, x, net), c2w, K, x_pix)

    for i in range(args.warmup):
        render(poses[i % len(poses)])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    fine_samples = 0
    t0 = time.perf_counter()
    frames = []
    for c2w in poses:
        rend.last_fine_samples = 0
        _, rgb_f, _, _ = render(c2w)
        fine_samples += getattr(rend, "last_fine_samples", 0)
        frames.append(rgb_f)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    secs = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([secs, float(fine_samples)], device=device, dtype=torch.float64)
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        secs, fine_samples = float(t[0]), int(t[1])
    if rank == 0:
        if args.out:
            os.makedirs(args.out, exist_ok=True)
            for i, f in enumerate(frames):
                write_ppm(os.path.join(args.out, f"frame_{i:03d}.ppm"), to_uint8(f[0].reshape(H, W, 3).cpu().numpy()))
        total_fine = args.frames * n * (args.n_coarse + args.n_fine)
        print(json.dumps({"renderer": args.renderer, "samples_per_ray": samples_per_ray,
                          "frames": args.frames, "res": args.res, "rays_per_frame": n, "n_gpus": world,
                          "seconds": round(secs, 4), "rays_per_s": round(args.frames * n / secs, 1),
                          "t_stop": args.t_stop, "precision": args.precision, "sigma_bias": args.sigma_bias,
                          "fine_samples_evaluated": fine_samples,
                          "fine_samples_fraction": round(fine_samples / total_fine, 4)}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
