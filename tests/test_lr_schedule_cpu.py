"""The graph-mode Trainer's per-epoch learning rate vs the reference scheduler: the reference steps
torch.optim.lr_scheduler.CosineAnnealingLR(T_max=1000, eta_min=1e-6) once per epoch
(baselightningmodule.py:80-92, interval "epoch"); the graph step keeps lr in a float64 device scalar that
Trainer.on_epoch_end rewrites (matcha/training.py) so the captured optimizer graph reads the new value."""
from __future__ import annotations

import pytest
import torch

from matcha.training import TrainConfig, Trainer


class _Tiny(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.w = torch.nn.Linear(4, 4)


@pytest.mark.filterwarnings("ignore:Detected call")
def test_graph_mode_cosine_matches_torch_scheduler():
    model = _Tiny()
    tr = Trainer(model, TrainConfig(graph=True))  # CPU: constructs the flat optimizer, launches nothing
    assert tr.scheduler is None and tr.lr.dtype == torch.float64
    ref_opt = torch.optim.AdamW(_Tiny().parameters(), lr=1e-4, betas=(0.9, 0.999), weight_decay=1e-6)
    ref = torch.optim.lr_scheduler.CosineAnnealingLR(ref_opt, T_max=1000, eta_min=1e-6)
    assert float(tr.lr) == ref.get_last_lr()[0] == 1e-4
    # through T_max (lr = eta_min at epoch 1000) and past it (the schedule is periodic in torch)
    for epoch in range(1, 2101):
        tr.on_epoch_end()
        ref.step()
        want = ref.get_last_lr()[0]
        got = float(tr.lr)
        assert abs(got - want) <= 1e-12 * max(abs(want), 1e-6) + 1e-18, (epoch, got, want)
    assert tr.epoch == 2100


@pytest.mark.filterwarnings("ignore:Detected call")
def test_eager_mode_uses_the_reference_scheduler():
    model = _Tiny()
    model.configure_optimizers = lambda: {  # BaseLightningClass.configure_optimizers on this stand-in
        "optimizer": (o := torch.optim.AdamW(model.parameters(), lr=1e-4, betas=(0.9, 0.999), weight_decay=1e-6)),
        "lr_scheduler": {"scheduler": torch.optim.lr_scheduler.CosineAnnealingLR(o, T_max=1000, eta_min=1e-6)}}
    tr = Trainer(model, TrainConfig(graph=False))
    for _ in range(3):
        tr.on_epoch_end()
    assert abs(tr.optimizer.param_groups[0]["lr"] - (1e-6 + (1e-4 - 1e-6) * (1 + torch.cos(torch.tensor(3 * torch.pi / 1000, dtype=torch.float64)).item()) / 2)) < 1e-15
