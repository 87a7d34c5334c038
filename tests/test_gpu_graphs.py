"""HIP-graph replay of the inference renderer (avr.graphs.GraphedRenderer): a replay with new cameras / pixels
equals the eager renderer on the same inputs and Philox offset bit for bit, and with the reference's torch
draws (seed None) the captured draws advance on every replay."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def _scene(R, seed):
    from avr.renderers import VolumeRenderer
    from avr.scene import INTRINSICS, synthetic_scene
    net = synthetic_scene(DEV, 0, latent_hw=(16, 16))
    g = torch.Generator(device="cpu").manual_seed(seed)
    x_pix = torch.rand(1, R, 2, generator=g).to(DEV)
    c2w = torch.eye(4).reshape(1, 1, 4, 4).repeat(1, R, 1, 1)
    c2w[..., 2, 3] = -1.3 - 0.2 * torch.rand(1, R, generator=g)
    K = torch.tensor([INTRINSICS], device=DEV)
    rend = VolumeRenderer(0.8, 1.8, 64, 32, 8, 0.01, True)
    return net, rend, c2w.to(DEV), K, x_pix


def test_graph_replay_equals_eager():
    from avr.graphs import GraphedRenderer
    net, rend, c2w, K, x_pix = _scene(1000, 1)
    rend.seed = 77
    gr = GraphedRenderer(rend, net, c2w, K, x_pix)
    for seed in (2, 3):
        _, _, c2w2, _, x2 = _scene(1000, seed)
        got = [t.clone() for t in gr(c2w2, K, x2)]
        rend._offset = gr.offset
        with torch.no_grad():
            want = rend(c2w2, K, x2, net)
        assert rend.last_path == "fused"
        for a, b in zip(got, want):
            assert torch.equal(a, b)


def test_graph_replay_torch_draws_advance():
    from avr.graphs import GraphedRenderer
    net, rend, c2w, K, x_pix = _scene(500, 4)
    rend.seed = None        # the reference's torch.rand / randn draws, captured with the graph
    gr = GraphedRenderer(rend, net, c2w, K, x_pix)
    a = [t.clone() for t in gr()]
    b = [t.clone() for t in gr()]
    assert all(bool(torch.isfinite(t).all()) for t in a + b)
    assert not torch.equal(a[1], b[1])          # new draws on every replay, as eager calls
    assert float((a[0] - b[0]).abs().mean()) < 0.05   # same scene: the coarse rgb moves by sampling noise only


def test_graph_recaptures_after_state_change():
    """An in-place weight update (an optimizer step) or a new latent (net.encode of new images) makes the next
    call capture the chain again, so the replay matches the eager renderer on the new state bit for bit."""
    from avr.graphs import GraphedRenderer
    net, rend, c2w, K, x_pix = _scene(300, 5)
    rend.seed = 11
    gr = GraphedRenderer(rend, net, c2w, K, x_pix)
    gr()
    gr()
    assert gr.captures == 1

    def check():
        got = [t.clone() for t in gr()]
        rend._offset = gr.offset
        with torch.no_grad():
            want = rend(c2w, K, x_pix, net)
        for a, b in zip(got, want):
            assert torch.equal(a, b)
        return got

    before = [t.clone() for t in gr()]
    with torch.no_grad():
        net.mlp_fine.lin_out.bias.add_(0.25)
    after = check()
    assert gr.captures == 2 and not torch.equal(before[1], after[1])
    net.encoder.set_latent(net.encoder.latent * 1.5)
    check()
    assert gr.captures == 3
    gr()
    assert gr.captures == 3


def test_graph_capture_and_replay_under_anomaly_mode():
    """torch anomaly mode (train.py --anomaly_detection) on: the warm-up calls are checked op by op, the capture
    skips the checks (a capture cannot synchronise), every replay checks its outputs; a clean scene raises
    nothing and the replay still equals the eager call."""
    from avr.graphs import GraphedRenderer
    net, rend, c2w, K, x_pix = _scene(300, 6)
    rend.seed = 5
    with torch.autograd.set_detect_anomaly(True):
        gr = GraphedRenderer(rend, net, c2w, K, x_pix)
        got = [t.clone() for t in gr()]
        rend._offset = gr.offset
        with torch.no_grad():
            want = rend(c2w, K, x_pix, net)
    for a, b in zip(got, want):
        assert torch.equal(a, b)


def _scenes(SB, R, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x_pix = torch.rand(SB, R, 2, generator=g).to(DEV)
    c2w = torch.eye(4).reshape(1, 1, 4, 4).repeat(SB, R, 1, 1)
    c2w[..., 2, 3] = -1.3 - 0.2 * torch.rand(SB, R, generator=g)
    return c2w.to(DEV), x_pix


def test_graph_survives_eager_calls_that_replace_caches():
    """the captured launches read FusedField's batched lin_z tables and packed blob. An eager call
    with another scene count replaces the batched-table cache entry, one at the other precision the packed
    entry; the graph keeps references to what it reads (and re-captures after a precision change), so the
    replay still equals the eager call. Capture and re-capture leave the renderer's Philox offset alone."""
    from avr.graphs import GraphedRenderer
    from avr.scene import INTRINSICS
    net, rend, _, _, _ = _scene(8, 1)
    net.encoder.set_latent(net.encoder.latent.expand(3, -1, -1, -1).contiguous() *
                           torch.tensor([1.0, 0.5, -1.0], device=DEV).reshape(3, 1, 1, 1))
    net.poses = net.poses.expand(3, 3, 4).contiguous()
    K = torch.tensor([INTRINSICS], device=DEV).expand(3, 3, 3).contiguous()
    rend.seed = 21
    c2w2, x2 = _scenes(2, 256, 7)
    gr = GraphedRenderer(rend, net, c2w2, K[:2], x2)
    assert rend._offset == 0 and gr.offset == 0
    c2w3, x3 = _scenes(3, 256, 8)
    with torch.no_grad():
        rend(c2w3, K, x3, net)                  # SB = 3: a new batched-table entry replaces the SB = 2 one
        net.field_precision = "fp32"
        rend(c2w2, K[:2], x2, net)              # the fp32 blob replaces the x3 one
        net.field_precision = "x3"
        torch.cuda.empty_cache()
        junk = torch.full((64 << 20,), float("nan"), device=DEV)   # reuse any freed block
    captures = gr.captures
    got = [t.clone() for t in gr()]
    assert gr.captures == captures              # back at x3: the capture's precision, no re-capture needed
    rend._offset = gr.offset
    with torch.no_grad():
        want = rend(c2w2, K[:2], x2, net)
    del junk
    for a, b in zip(got, want):
        assert torch.equal(a, b)
    net.field_precision = "fp32"
    gr()
    assert gr.captures == captures + 1          # a precision change re-captures
    net.field_precision = "x3"


@pytest.mark.parametrize("side", ["1", "0"])
def test_graphed_train_step_matches_eager_adaptive(side, monkeypatch):
    """avr.graphs.GraphedTrainStep: bench.run_train's AdaptiveVolumeRenderer train.py step (default_mv field,
    4 scenes x 512 rays, capturable fused Adam) captured once and replayed gives the eager step's losses and parameters
    bit for bit over several steps -- the CPU start distances staged per replay draw the same values, the band's
    device draws advance as eager ones do -- with the marched point's pass on its side stream inside the graph or
    not."""
    from test_gpu_poison import _setup
    from avr.graphs import GraphedTrainStep
    monkeypatch.setenv("AVR_ADAPTIVE_SIDE_STREAM_IN_GRAPH", side)
    runs = []
    for graphed in (False, True):
        net, rend, named, (c2w, K, x_pix, gt), _ = _setup("adaptive", False)
        opt = torch.optim.Adam([p for _, p in named], lr=1e-4, capturable=True, fused=True)

        def step():
            rgb_c, rgb_f, _, _ = rend(c2w, K, x_pix, net)
            loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
            opt.zero_grad()
            loss.backward()
            opt.step()
            return loss
        run = GraphedTrainStep(step, nets=[net], renderers=[rend], warmup=2) if graphed else step
        torch.manual_seed(123)
        losses = [float(run()) for _ in range(6)]
        assert rend.last_path == "hip_train"
        if graphed:
            assert run.captures == 1 and run.calls == 6
        runs.append((losses, {n: p.detach().clone() for n, p in named}))
    (le, pe), (lg, pg) = runs
    assert all(torch.isfinite(torch.tensor(le)))
    assert le == lg, (le, lg)
    for n in pe:
        assert torch.equal(pe[n], pg[n]), n


def test_graphed_train_step_recaptures_after_view_change():
    """GraphedTrainStep with new source views between steps (poses updated in place, as a new batch of scenes
    would): the call that sees the change runs eagerly (it rebuilds the host-side view descriptors), the next
    one captures again, and every step's loss equals the eager run's with the same change."""
    from test_gpu_poison import _setup
    from avr.graphs import GraphedTrainStep
    runs = []
    for graphed in (False, True):
        net, rend, named, (c2w, K, x_pix, gt), _ = _setup("adaptive", False)
        opt = torch.optim.Adam([p for _, p in named], lr=1e-4, capturable=True, fused=True)

        def step():
            rgb_c, rgb_f, _, _ = rend(c2w, K, x_pix, net)
            loss = ((rgb_c - gt) ** 2).mean() + ((rgb_f - gt) ** 2).mean()
            opt.zero_grad()
            loss.backward()
            opt.step()
            return loss
        run = GraphedTrainStep(step, nets=[net], renderers=[rend], warmup=1) if graphed else step
        torch.manual_seed(321)
        losses = []
        for i in range(7):
            if i == 4:
                with torch.no_grad():
                    net.poses[:, 0, 3] += 0.02      # new source views, same shapes
            losses.append(float(run()))
        if graphed:
            assert run.captures == 2, run.captures
        runs.append(losses)
    assert runs[0] == runs[1], runs
