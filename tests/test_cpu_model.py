"""Drop-in module API on CPU (no kernels are launched): state_dict keys/shapes, parameter
counts and .parameters() order equal the reference's (modules/model.py:90-131; counts from
SURVEY.md §8b), the checkpoint interchange format, and the no-CPU-fallback rule."""
import pytest
import torch

from oracle import ref_torch as orc


@pytest.mark.parametrize("cin,nb,cbam,count", [(3, 9, True, 11_446_515), (1, 9, True, 11_440_243),
                                               (2, 9, True, None), (1, 2, False, None)])
def test_generator_state_dict_layout(cin, nb, cbam, count):
    from modules.model import Generator
    G = Generator(input_channels=cin, num_residual_blocks=nb, use_cbam=cbam)
    want = orc.generator_param_shapes(cin, nb, cbam)
    got = {k: tuple(v.shape) for k, v in G.state_dict().items()}
    assert list(got) == list(want)           # same keys in the same order (no IN buffers)
    assert got == want
    assert [n for n, _ in G.named_parameters()] == list(want)  # optimizer index order
    if count is not None:
        assert sum(p.numel() for p in G.parameters()) == count


def test_discriminator_state_dict_layout():
    from modules.model import Discriminator
    D = Discriminator()
    want = orc.discriminator_param_shapes(1)
    assert {k: tuple(v.shape) for k, v in D.state_dict().items()} == want
    assert [n for n, _ in D.named_parameters()] == list(want)
    assert sum(p.numel() for p in D.parameters()) == 2_762_689


def test_weights_init_normal():
    from modules.model import Generator, weights_init_normal
    torch.manual_seed(0)
    G = Generator(3, 2)
    G.apply(weights_init_normal)
    w = G.model[10].block[1].weight
    w = w.detach()
    assert abs(float(w.mean())) < 1e-3 and abs(float(w.std()) - 0.02) < 1e-3
    b = G.model[1].bias  # biases keep torch's default U(+-1/sqrt(fan_in))
    assert float(b.abs().max()) <= 1 / (3 * 49) ** 0.5


def test_reference_checkpoint_roundtrip(tmp_path):
    """A reference-layout G checkpoint (plain or DataParallel 'module.'-prefixed state_dict)
    saved with torch.save loads into the drop-in Generator with the weights-only loader."""
    from modules.model import Generator
    G = Generator(3, 1)
    sd = {k: torch.randn(v.shape) for k, v in G.state_dict().items()}
    path = tmp_path / "G_A2B_last.pth"
    torch.save(sd, path)
    G2 = Generator(3, 1)
    G2.load_state_dict(torch.load(path, weights_only=True))
    for k, v in G2.state_dict().items():
        assert torch.equal(v, sd[k])


def test_no_cpu_fallback():
    """The product forward needs device tensors: a CPU input raises instead of computing."""
    from modules.model import Discriminator, Generator
    with pytest.raises((RuntimeError, AssertionError)):
        Generator(3, 1)(torch.zeros(1, 3, 16, 16))
    with pytest.raises((RuntimeError, AssertionError)):
        Discriminator()(torch.zeros(1, 1, 32, 32))
