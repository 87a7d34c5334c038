import torch
dev = torch.device("cuda:0")
for mb in (33.5, 134, 536):
    n = int(mb * 1e6 / 4)
    x = torch.empty(n, device=dev); y = torch.empty(n, device=dev)
    for name, fn in (("fill", lambda: x.fill_(1.0)), ("zero", lambda: x.zero_()), ("copy", lambda: x.copy_(y))):
        fn(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50): fn()
        e1.record(); torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 50
        nb = n * 4 * (2 if name == "copy" else 1)
        print(f"{mb} MB {name}: {us:.1f} us {nb / us / 1e3:.0f} GB/s", flush=True)
