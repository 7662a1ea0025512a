"""Whole-network numerics: the native engine (BN folded, bf16, hand-written
kernels) against the fp32 PyTorch oracle (BN unfused) on the same random-init
weights. Compared on logits/probabilities (random-init top-5 is ill-conditioned,
SURVEY §4 item 4)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from distributed_machine_learning_amd.models import build_model  # noqa: E402
from distributed_machine_learning_amd.models.engine import Engine  # noqa: E402
from distributed_machine_learning_amd.models.oracle import OracleExecutor, preprocess_reference  # noqa: E402


@pytest.mark.parametrize("name", ["ResNet50", "InceptionV3"])
def test_engine_matches_oracle(name):
    g, w = build_model(name, seed=0, calibrate=True)
    torch.manual_seed(0)
    hw = g.input_hw
    imgs = torch.randint(0, 256, (2, hw[0], hw[1], 3), dtype=torch.uint8)
    eng = Engine(g, w, batch=2)
    eng.infer(imgs.cuda())
    torch.cuda.synchronize()
    ref = OracleExecutor(g, w).forward(preprocess_reference(imgs, hw, g.preprocess))
    got = eng.buf[g.logits].float().cpu()
    rl = ref["logits"]
    rel = ((got - rl).abs().max() / rl.abs().max()).item()
    assert rel < 5e-2, rel
    # softmax probabilities close
    assert (eng.probs.cpu() - ref["probs"]).abs().max().item() < 5e-2
    # top-1 agrees where the oracle has a clear winner
    rv, ri = ref["probs"].topk(2, dim=-1)
    clear = (rv[:, 0] - rv[:, 1]) > 0.05
    assert torch.equal(eng.top_idx.cpu()[clear, 0].long(), ri[clear, 0])


def test_graph_replay_matches_eager():
    g, w = build_model("ResNet50", seed=1, calibrate=False)
    eng = Engine(g, w, batch=4)
    imgs = torch.randint(0, 256, (4, 224, 224, 3), dtype=torch.uint8, device="cuda")
    eng.src.copy_(imgs)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        eng.run(s)
        s.synchronize()
        eager = eng.buf[g.logits].clone()
        eng.buf[g.logits].zero_()
        eng.run(s, use_graph=True)
        s.synchronize()
    assert torch.equal(eager, eng.buf[g.logits])


def test_batch_rows_independent():
    """Row i of a batch-4 run equals the batch-1 run of image i (no cross-image leakage)."""
    g, w = build_model("ResNet50", seed=2, calibrate=False)
    imgs = torch.randint(0, 256, (4, 224, 224, 3), dtype=torch.uint8, device="cuda")
    e4 = Engine(g, w, batch=4)
    e1 = Engine(g, w, batch=1)
    e4.infer(imgs)
    outs = []
    for i in range(4):
        e1.infer(imgs[i:i + 1])
        torch.cuda.synchronize()
        outs.append(e1.buf[g.logits].clone())
    torch.cuda.synchronize()
    assert torch.allclose(torch.cat(outs), e4.buf[g.logits], atol=1e-3, rtol=1e-3)
