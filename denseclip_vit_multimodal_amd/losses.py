"""SILog depth loss (reference seg/denseclip/losses.py:7-78)."""
import torch
import torch.nn as nn


class SILogLoss(nn.Module):
    def __init__(self, lambd=0.5, eps=1e-6, reduction="mean"):
        super().__init__()
        if reduction not in ("mean", "sum"):
            raise ValueError(f"Invalid reduction type: {reduction}. Must be 'mean' or 'sum'.")
        self.lambd = lambd
        self.eps = eps
        self.reduction = reduction

    def forward(self, prediction, target, mask=None):
        d = torch.log(torch.clamp(prediction, min=self.eps)) - torch.log(torch.clamp(target, min=self.eps))
        if mask is not None:
            if mask.shape != d.shape:
                if mask.dim() == d.dim() - 1:
                    mask = mask.unsqueeze(1)
                else:
                    raise ValueError(f"Mask shape {mask.shape} incompatible with log_diff shape {d.shape}")
            d = torch.where(mask, d, torch.zeros_like(d))
            T = mask.sum()
        else:
            T = torch.tensor(float(d.numel()), device=d.device)
        # T as a device tensor: no host sync (the reference calls .item() here)
        Tf = T.to(d.dtype).clamp(min=1)
        loss = (d ** 2).sum() / Tf - self.lambd * d.sum() ** 2 / Tf ** 2
        return torch.where(T > 0, loss, torch.zeros_like(loss))
