"""Checkpoint compatibility and host data path (8f row 4)."""
import collections
import os

import numpy as np
import pytest
import torch


def _small_model():
    from image_compression_amd import get_cfg_defaults, modelling
    cfg = get_cfg_defaults()
    cfg.MODEL.INTER_CHANNELS = 16
    cfg.MODEL.LATENT_CHANNELS = 16
    return modelling.build_model(cfg)


def test_reference_checkpoint_loads(tmp_path):
    """A checkpoint in the reference's layout (DataParallel "module." keys,
    torch AdamW + LambdaLR state, iter, best_metric) loads into our model and
    optimizer, via a loader that never unpickles code."""
    from image_compression_amd.checkpoint import add_prefix, load_file, load_model_weights
    from image_compression_amd.solver import AdamW
    torch.manual_seed(1)
    src = _small_model()
    opt = torch.optim.AdamW([{"params": [p], "lr": 1e-4, "weight_decay": 5e-4} for p in src.parameters()],
                            1e-4, eps=1e-4)
    for p in src.parameters():
        p.grad = torch.randn_like(p)
    opt.step()
    sch = torch.optim.lr_scheduler.LambdaLR(opt, lambda _: 1)
    cp = {"state_dict": add_prefix(src.state_dict()), "optimizer": opt.state_dict(),
          "scheduler": sch.state_dict(), "iter": 7, "best_metric": 28.868}
    path = os.path.join(tmp_path, "iter_00000007_28.8680.pth")
    torch.save(cp, path)
    torch.manual_seed(2)
    dst = _small_model()
    load_model_weights(dst, path)
    for (k, a), (k2, b) in zip(src.state_dict().items(), dst.state_dict().items()):
        assert k == k2 and torch.equal(a, b), k
    ours = AdamW([{"params": [p], "lr": 1e-4, "weight_decay": 5e-4} for p in dst.parameters()], 1e-4, eps=1e-4)
    ours.load_state_dict(load_file(path)["optimizer"])
    st = ours.state[next(iter(dst.parameters()))]
    assert int(st["step"]) == 1 and st["exp_avg"].shape == next(iter(dst.parameters())).shape


def test_iter_checkpointer_rotation_and_resume(tmp_path):
    from image_compression_amd.checkpoint import IterCheckpointer, load_file
    model = _small_model()
    ck = IterCheckpointer(str(tmp_path), model, num_checkpoints=2)
    ck.save_checkpoint(True, iter=1, current_metric=20.0)
    ck.save_checkpoint(False, iter=2)
    ck.save_checkpoint(True, iter=3, current_metric=25.0)
    files = sorted(os.listdir(os.path.join(tmp_path, "checkpoints")))
    assert "iter_00000001.pth" not in files                      # rotated out
    assert {"iter_00000002.pth", "iter_00000003.pth", "iter_00000003_25.0000.pth",
            "checkpoints_logs.json"} <= set(files)
    assert "iter_00000001_20.0000.pth" not in files               # superseded best
    cp = load_file(os.path.join(tmp_path, "checkpoints", "iter_00000003.pth"))
    assert all(k.startswith("module.") for k in cp["state_dict"])  # loadable by the reference
    assert cp["iter"] == 3 and cp["best_metric"] == 25.0
    ck2 = IterCheckpointer(str(tmp_path), _small_model(), num_checkpoints=2)
    assert ck2.load_resume() == 4


def test_random_crop_and_sampler_follow_reference_rng(tmp_path):
    from PIL import Image
    from image_compression_amd.data import ImageNetDataset, KodakDataset, TrainingSampler, collate
    rng = np.random.RandomState(0)
    for i in range(3):
        Image.fromarray(rng.randint(0, 256, (40, 50, 3), dtype=np.uint8)).save(os.path.join(tmp_path, f"im{i}.png"))
    meta = os.path.join(os.path.dirname(tmp_path), "meta.csv")   # outside the image folder (Kodak globs it all)
    with open(meta, "w") as f:
        f.write("path\n" + "\n".join(f"im{i}.png" for i in range(3)) + "\n")
    ds = ImageNetDataset(str(tmp_path), meta, "train", crop=16)
    np.random.seed(5)
    ident, crop = ds[1]
    np.random.seed(5)                                  # the reference's draws: x then y
    x, y = np.random.randint(50 - 16 + 1), np.random.randint(40 - 16 + 1)
    full = np.asarray(Image.open(os.path.join(tmp_path, "im1.png")).convert("RGB"))
    assert crop.shape == (16, 16, 3) and crop.dtype == torch.uint8
    assert np.array_equal(crop.numpy(), full[y:y + 16, x:x + 16])
    kd = KodakDataset(str(tmp_path))
    assert [kd[i][0] for i in range(len(kd))] == ["im0", "im1", "im2"] and kd[0][1].shape == (40, 50, 3)
    it = iter(TrainingSampler(3, True, seed=4))
    g = torch.Generator()
    g.manual_seed(4)
    want = torch.randperm(3, generator=g).tolist() + torch.randperm(3, generator=g).tolist()
    assert [next(it) for _ in range(6)] == want
    b = collate([ds[0], ds[2]])
    assert b.imgs.shape == (2, 16, 16, 3)


@pytest.mark.gpu
def test_device_input_conversion_matches_reference_transform():
    from image_compression_amd.data import to_device_input
    rng = np.random.RandomState(1)
    u8 = torch.from_numpy(rng.randint(0, 256, (2, 24, 36, 3), dtype=np.uint8))
    mean, std = (0.1, 0.2, 0.3), (0.9, 0.8, 0.7)
    y = to_device_input(u8, "cuda", mean, std).cpu()
    ref = (u8.float().permute(0, 3, 1, 2) / 255.0 - torch.tensor(mean).view(1, 3, 1, 1)) / torch.tensor(std).view(1, 3, 1, 1)
    assert torch.allclose(y, ref, rtol=1e-6, atol=1e-7)
    y0 = to_device_input(u8, "cuda").cpu()
    assert torch.equal(y0, u8.float().permute(0, 3, 1, 2) / 255.0)


def test_colsum_handoff_is_keyed_by_the_gradient_itself():
    """functional._put_colsum / _take_colsum: a stashed column sum is handed only to the very
    gradient tensor it was formed from, unchanged since (version counter), and only once."""
    import torch
    from image_compression_amd import functional as IF
    t, s = torch.zeros(4, 3), torch.ones(3)
    IF._put_colsum(t, s)
    assert IF._take_colsum(torch.zeros(4, 3)) is None      # another tensor
    IF._put_colsum(t, s)
    assert IF._take_colsum(t) is s and IF._take_colsum(t) is None   # once
    IF._put_colsum(t, s)
    t.add_(1.0)                                               # changed after the sums were formed
    assert IF._take_colsum(t) is None
