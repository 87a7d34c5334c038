"""Does a captured step with Adam(capturable=True, fused=True) match eager steps on this torch / ROCm? (probe)"""
import torch

for fused in (False, True):
    res = []
    for graphed in (False, True):
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.ReLU(), torch.nn.Linear(64, 1)).cuda()
        x = torch.randn(256, 64, device="cuda")
        y = torch.randn(256, 1, device="cuda")
        opt = torch.optim.Adam(m.parameters(), lr=1e-2, capturable=True, fused=fused)

        def step():
            loss = ((m(x) - y) ** 2).mean()
            opt.zero_grad()
            loss.backward()
            opt.step()
            return loss.detach()
        losses = []
        if graphed:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    losses.append(float(step()))
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                out = step()
            for _ in range(4):
                g.replay()
                losses.append(float(out))
        else:
            losses = [float(step()) for _ in range(6)]
        res.append(losses)
    print(f"fused={fused}: eager {res[0]}\n            graph {res[1]}\n            equal {res[0] == res[1]}")
