"""The reference's helper functions are callable with the reference's own arguments
(``/root/reference/singlegpu.py:132`` ``load_train_objs()``, ``:174`` ``prepare_dataloader(dataset, batch_size)``,
``multigpu.py:125`` / ``:147`` likewise) while the ddpx-extended forms keep working."""
import importlib
import sys

import pytest
import torch


@pytest.mark.parametrize("entry", ["singlegpu", "multigpu"])
def test_reference_signatures(entry, monkeypatch):
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)  # CPU box: resolve to the CPU
    mod = importlib.import_module(entry)
    from ddpx.train import app
    cfg = app.build_parser("t").parse_args(["2", "1", "--train_size", "512", "--test_size", "128", "--data",
                                            "synthetic"])
    app.set_config(cfg)
    try:
        train_set, model, optimizer, test_set, scheduler = mod.load_train_objs()
        assert len(train_set) == 512 and len(test_set) == 128
        assert type(model).__name__ == "VGG"
        g = optimizer.param_groups[0]
        assert (g["momentum"], g["weight_decay"]) == (0.9, 5e-4)
        assert scheduler.get_last_lr()[0] == 0.0  # one-cycle starts at lr 0
        loader = mod.prepare_dataloader(train_set, 64)
        assert len(loader) == 8
        x, y = next(iter(loader))
        assert x.shape == (64, 3, 32, 32) and x.dtype == torch.float32 and y.shape == (64,)
        assert 0.0 <= float(x.min()) and float(x.max()) <= 1.0
    finally:
        app.set_config(None)


def test_default_config_is_the_reference_recipe():
    from ddpx.train import app
    app.set_config(None)
    cfg = app.current_config()
    assert (cfg.total_epochs, cfg.save_every, cfg.batch_size, cfg.model, cfg.lr) == (20, 5, 512, "vgg", 0.4)
    app.set_config(None)
