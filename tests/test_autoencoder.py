"""Frame encoder / decoder CNNs and the autoencoder loss (model/models.py:10-117,
losses.py:5-16) against the reference's own outputs
(tests/golden/autoencoder.npz).  These are per-frame (B x T images) PyTorch/MIOpen work, not
particle work: same layers, same construction order, so the same seed gives the reference's
parameters (checked by per-parameter checksums); outputs are compared on the CPU and, on the
GPU box, through MIOpen."""
import numpy as np
import pytest
import torch

from _util import group, load

CASES = [("h32", "build_encoder", "build_decoder", 32), ("cglow", "build_encoder_cglow", "build_decoder_cglow", 192)]


def _build(tag, benc, bdec, H):
    import model.models as mm
    torch.manual_seed(301)
    enc = getattr(mm, benc)(H)
    torch.manual_seed(302)
    dec = getattr(mm, bdec)(H)
    return enc, dec


def _check(tag, benc, bdec, H, device, rtol, atol):
    from losses import autoencoder_loss
    fx = group(load("autoencoder.npz"), tag)
    enc, dec = _build(tag, benc, bdec, H)
    for name, m in (("enc", enc), ("dec", dec)):
        sd = m.state_dict()
        keys = {k[len(name) + 5:] for k in fx if k.startswith(f"{name}/sum/")}
        assert keys == set(sd), (sorted(keys ^ set(sd)))
        for k, v in sd.items():
            assert float(v.double().sum()) == pytest.approx(float(fx[f"{name}/sum/{k}"]), rel=1e-9, abs=1e-9), k
            assert float(v.double().abs().sum()) == pytest.approx(float(fx[f"{name}/abs/{k}"]), rel=1e-9), k
    enc, dec = enc.to(device), dec.to(device)
    g = torch.Generator().manual_seed(303)
    img = torch.rand(2, 2, 3, 128, 128, generator=g)
    idx = torch.randint(0, 4 * 3 * 128 * 128, (512,), generator=g)
    np.testing.assert_array_equal(idx.numpy(), fx["idx"])
    img = img.to(device)
    for mode in ("train", "eval"):
        enc.train(mode == "train")
        dec.train(mode == "train")
        with torch.no_grad():
            f = enc(img.reshape(4, 3, 128, 128))
            r = dec(f)
            loss = autoencoder_loss(img, mode == "train", enc, dec)
        np.testing.assert_allclose(f.cpu().numpy(), fx[f"{mode}/feature"], rtol=rtol, atol=atol)
        np.testing.assert_allclose(r.reshape(-1)[idx.to(device)].cpu().numpy(), fx[f"{mode}/recon_sample"],
                                   rtol=rtol, atol=atol)
        np.testing.assert_allclose(r.mean(dim=(0, 2, 3)).cpu().numpy(), fx[f"{mode}/recon_mean"], rtol=rtol,
                                   atol=atol)
        assert float(loss) == pytest.approx(float(fx[f"{mode}/loss"]), rel=10 * rtol, abs=atol)


@pytest.mark.parametrize("tag,benc,bdec,H", CASES)
def test_autoencoder_cpu(tag, benc, bdec, H):
    _check(tag, benc, bdec, H, torch.device("cpu"), 1e-5, 1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("tag,benc,bdec,H", CASES)
def test_autoencoder_gpu(tag, benc, bdec, H):
    # MIOpen convolutions (different algorithms / accumulation order from the CPU's oneDNN)
    _check(tag, benc, bdec, H, torch.device("cuda:0"), 2e-4, 2e-5)
