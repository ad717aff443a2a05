"""Training hooks of the reference's BaseLightningClass (matcha/models/baselightningmodule.py:19-246)
without pytorch_lightning (not part of this stack): the same get_losses / training_step /
configure_optimizers semantics, driven by matcha.training.Trainer instead of Lightning's loop.
"""
from __future__ import annotations

from typing import Any

import torch
import torch.nn as nn


class BaseLightningClass(nn.Module):
    global_step: int = 0

    def update_data_statistics(self, data_statistics):
        if data_statistics is None:
            data_statistics = {"mel_mean": 0.0, "mel_std": 1.0}
        self.register_buffer("mel_mean", torch.tensor(data_statistics["mel_mean"]))
        self.register_buffer("mel_std", torch.tensor(data_statistics["mel_std"]))

    def save_hyperparameters(self, *args, **kwargs):  # Lightning API kept as a no-op
        pass

    def log(self, name, value, **kwargs):  # Lightning API: recorded for the driver to reduce/print
        self.__dict__.setdefault("_logged", {})[name] = value

    def configure_optimizers(self) -> dict[str, Any]:
        """baselightningmodule.py:57-92: AdamW(1e-4, (0.9, 0.999), wd 1e-6) + per-epoch cosine
        annealing (T_max 1000, eta_min 1e-6)."""
        # torch's default implementation, as the reference (multi-tensor on the GPU); the graph-mode
        # Trainer replaces it with the HIP clip + AdamW, equal to it within 2 ulp
        opt = torch.optim.AdamW(self.parameters(), lr=1e-4, betas=(0.9, 0.999), weight_decay=1e-6)
        sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=1000, eta_min=1e-6)
        return {"optimizer": opt, "lr_scheduler": {"scheduler": sched, "interval": "epoch", "frequency": 1}}

    def get_losses(self, batch):
        """baselightningmodule.py:94-110."""
        dur_loss, prior_loss, diff_loss, *_ = self(
            x=batch["x"], x_lengths=batch["x_lengths"], y=batch["y"], y_lengths=batch["y_lengths"],
            out_size=self.out_size, durations=batch.get("durations", None))
        return {"dur_loss": dur_loss, "prior_loss": prior_loss, "diff_loss": diff_loss}

    def training_step(self, batch: Any, batch_idx: int):
        """baselightningmodule.py:115-162: total = dur + prior + diff."""
        loss_dict = self.get_losses(batch)
        total = sum(loss_dict.values())
        self.log("loss/train", total)
        return {"loss": total, "log": loss_dict}
