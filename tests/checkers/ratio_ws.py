"""Readers of the ratio predictor's workspace diagnostics (include/rgbd_hip.h
`rgbd_ratio_features_offset`): the bf16 gated features sit in conv5 v4's input layout, channel
quarters in zero-padded planes [B][4][PH][PW][32] with pixel (y, x) at (y + 1, x + 1),
PH = ceil(H / 16) * 16 + 2, PW = ceil(W / 32) * 32 + 2."""


def ratio_features_bf16(ws, off, B, H, W):
    """[B, 128, H, W] bf16 view-copy of the gated features from a uint8 workspace tensor."""
    import torch
    PH, PW = -(-H // 16) * 16 + 2, -(-W // 32) * 32 + 2
    n = B * 4 * PH * PW * 32
    planes = ws[off:off + 2 * n].view(torch.bfloat16).reshape(B, 4, PH, PW, 32)
    return planes[:, :, 1:H + 1, 1:W + 1].permute(0, 1, 4, 2, 3).reshape(B, 128, H, W)


def ratio_pad_is_zero(ws, off, B, H, W):
    """True when every padding element of the bf16 feature planes is +0 (bitwise)."""
    import torch
    PH, PW = -(-H // 16) * 16 + 2, -(-W // 32) * 32 + 2
    n = B * 4 * PH * PW * 32
    planes = ws[off:off + 2 * n].view(torch.int16).reshape(B, 4, PH, PW, 32)
    mask = torch.ones((PH, PW), dtype=torch.bool, device=planes.device)
    mask[1:H + 1, 1:W + 1] = False
    return bool((planes[:, :, mask] == 0).all())
