"""Drop-in nn.Modules for the reference's hot-path sub-operators.

Same constructor signatures, forward signatures, parameter names (state_dict keys) and
error behaviour as the reference classes in mask2former/utils/custom_model.py; the compute
runs in librgbd_hip.so.

  DSAModule(in_channels, out_channels, num_depth_regions=3)              (:622-798)
  DepthGradientInjectionResidual(color_channels, depth_gradient_channels) (:1169-1269)
  EnhancedDepthImageRatioPredictor(input_channels=3)                     (:1363-1487)
"""
import numpy as np
import torch
from torch import nn

from . import ops
from .hot_path import stack4


class _DSAMFn(torch.autograd.Function):
    """One DSAModule over a batch of features sharing ``code``/``info`` (decomposed outside)."""

    @staticmethod
    def forward(ctx, x, code, info, dtype, pack_cache, *params):
        conv_ws, biases, proj_w = params[0:8:2], params[1:8:2], params[8]
        xc = x.detach().to(dtype)
        x_nhwc = ops.nchw_to_nhwc(xc.contiguous())
        training = any(ctx.needs_input_grad[5:])
        mask = ops.dsam_code_masks([code]) if dtype == torch.bfloat16 else None
        wfwd, wbwd = pack_cache.get(conv_ws, proj_w, dtype, code_mask=mask, want_bwd=training)
        out, _ = ops.dsam_fwd(x_nhwc, code, info, wfwd, stack4([b.detach() for b in biases]))
        ctx.save_for_backward(x_nhwc, code, info, wbwd)
        ctx.cin = x.shape[1]
        ctx.x_dtype = x.dtype
        return out.to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        x_nhwc, code, info, wbwd = ctx.saved_tensors
        g = g.to(x_nhwc.dtype).contiguous()
        g_nhwc = ops.nchw_to_nhwc(g)
        dconv, dproj, dbias = ops.dsam_bwd_weight(g, x_nhwc, code, info, gout_nhwc=g_nhwc)
        dx = None
        if ctx.needs_input_grad[0]:
            dx, _ = ops.dsam_bwd_data(g_nhwc, code, wbwd, None, cin=ctx.cin)
            dx = dx.to(ctx.x_dtype)
        grads = []
        for i in range(4):
            grads += [dconv[i], dbias[i]]
        grads.append(dproj)
        return (dx, None, None, None, None, *grads)


class DSAModule(nn.Module):
    """Depth-Sensitive Attention Module (reference custom_model.py:622-699).

    ``compute_dtype`` (float32 | bfloat16) selects the MFMA precision; the depth
    decomposition is always float32."""

    def __init__(self, in_channels, out_channels, num_depth_regions=3):
        super().__init__()
        if in_channels == out_channels:
            raise NotImplementedError("v0.4.0 only instantiates DSAModule with in != out channels "
                                      "(custom_model.py:129-131); the 1x1 variant is out of scope")
        if num_depth_regions != 3:
            raise NotImplementedError("num_depth_regions is fixed to 3 by v0.4.0")
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.num_depth_regions = num_depth_regions
        self.conv_layers = nn.ModuleList([
            nn.Conv2d(in_channels, out_channels, kernel_size=3, stride=2, padding=1)
            for _ in range(num_depth_regions + 1)])
        self.rgb_projection = nn.Conv2d(in_channels, out_channels, kernel_size=3, stride=2, padding=1,
                                        bias=False)
        self.compute_dtype = torch.float32
        from .hot_path import _PackCache
        self._pack_cache = _PackCache()
        self._group_storage()

    def _group_storage(self):
        """Keep the four conv_layers weights (and the four biases) in one storage each, in order,
        so the packer and the fused forward read them as the [4, ...] arrays they take
        (hot_path.stack4 then returns a view instead of copying 2 x 4 tensors every step).
        Parameter identity is kept (only .data moves), so optimizers and state_dicts are
        unaffected; re-applied after every .to() / .cuda() (Module._apply)."""
        from .hot_path import stack4
        with torch.no_grad():
            for attr in ("weight", "bias"):
                ps = [getattr(self.conv_layers[i], attr) for i in range(4)]
                if stack4([p.data for p in ps], view_only=True) is not None:
                    continue
                flat = torch.stack([p.data for p in ps])
                for i, p in enumerate(ps):
                    p.data = flat[i]

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._group_storage()
        return out

    def _params(self):
        p = []
        for i in range(4):
            p += [self.conv_layers[i].weight, self.conv_layers[i].bias]
        p.append(self.rgb_projection.weight)
        return p

    def forward(self, rgb_features, depth_map, window_size_ratio=0.1):
        """rgb_features [B,Cin,h,w]; depth_map: grey depth tensor [H,W] / [1,H,W] / [B,1,H,W]
        (or numpy); window_size_ratio: float or per-image tensor.  (:647-699)"""
        if isinstance(depth_map, np.ndarray):
            depth_map = torch.from_numpy(np.ascontiguousarray(depth_map)).to(rgb_features.device)
        elif not isinstance(depth_map, torch.Tensor):
            raise TypeError("Depth map must be torch.Tensor or numpy.ndarray")
        B = rgb_features.shape[0]
        d = depth_map.float()
        while d.dim() < 4:
            d = d.unsqueeze(0)
        if d.shape[0] == 1 and B > 1:
            d = d.expand(B, -1, -1, -1)
        d = d.reshape(B, 1, d.shape[-2], d.shape[-1]).contiguous()
        if isinstance(window_size_ratio, torch.Tensor):
            r = window_size_ratio.detach().float().reshape(-1).to(d.device)
            r = r.expand(B).contiguous() if r.numel() == 1 else r
        else:
            r = torch.full((B,), float(window_size_ratio), dtype=torch.float32, device=d.device)
        h, w = rgb_features.shape[2:]
        codes, info = ops.edsam_decompose(d, r, [(h, w)])
        ops.raise_on_status(info)
        return _DSAMFn.apply(rgb_features, codes[0], info, self.compute_dtype, self._pack_cache, *self._params())


class _DGGMFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, color, planes, dtype, weight, bias):
        c = color.detach().to(dtype).contiguous()
        out = ops.dggm_fuse_fwd(None, c, planes, weight.detach(), bias.detach())
        ctx.save_for_backward(planes, weight, bias)
        ctx.dtypes = (color.dtype, dtype)
        return out.to(color.dtype)

    @staticmethod
    def backward(ctx, g):
        planes, weight, bias = ctx.saved_tensors
        dw, db = ops.dggm_fuse_bwd(g.to(ctx.dtypes[1]).contiguous(), planes, weight.detach(), bias.detach())
        return g, None, None, dw.reshape(weight.shape), db


class DepthGradientInjectionResidual(nn.Module):
    """Gated depth-gradient residual injection (reference custom_model.py:1169-1269)."""

    def __init__(self, color_channels, depth_gradient_channels):
        super().__init__()
        self.color_channels = color_channels
        self.depth_gradient_channels = depth_gradient_channels
        self.num_scales = len(color_channels)
        self.depth_enhancement_layers = nn.ModuleList()
        for channels in color_channels:
            self.depth_enhancement_layers.append(nn.Sequential(
                nn.Conv2d(depth_gradient_channels, channels, kernel_size=1), nn.ReLU(inplace=True)))
        self.compute_dtype = torch.float32

    def forward(self, color_feature_maps, processed_depth_gradient_map, gradient_mask):
        assert len(color_feature_maps) == self.num_scales, \
            f"Expected {self.num_scales} color feature maps, but got {len(color_feature_maps)}"
        if processed_depth_gradient_map is None or gradient_mask is None:
            return list(color_feature_maps)  # passthrough (:1263-1265)
        assert processed_depth_gradient_map.shape[1] == self.depth_gradient_channels
        assert gradient_mask.shape[1] == 1
        if self.depth_gradient_channels != 3:
            raise NotImplementedError("the HIP gate is specialised for 3 gradient channels (v0.4.0)")
        planes = torch.cat([processed_depth_gradient_map, gradient_mask], dim=1).float().contiguous()
        out = []
        for i, c in enumerate(color_feature_maps):
            conv = self.depth_enhancement_layers[i][0]
            out.append(_DGGMFn.apply(c, planes, self.compute_dtype, conv.weight, conv.bias))
        return out


class EnhancedDepthImageRatioPredictor(nn.Module):
    """Window-size-ratio predictor (reference custom_model.py:1363-1487).  Same module tree /
    state_dict keys; the forward runs the HIP ratio-predictor pipeline (ratio.py)."""

    def __init__(self, input_channels: int = 3):
        super().__init__()
        self.input_channels = input_channels

        def cbr(cin, cout, k):
            return nn.Sequential(nn.Conv2d(cin, cout, kernel_size=k, padding=k // 2), nn.BatchNorm2d(cout),
                                 nn.ReLU(inplace=True))
        self.scale1_conv = cbr(input_channels, 64, 3)
        self.scale2_conv = cbr(input_channels, 64, 5)
        self.scale3_conv = cbr(input_channels, 64, 7)
        self.feature_fusion = nn.Sequential(nn.Conv2d(192, 128, kernel_size=1), nn.BatchNorm2d(128),
                                            nn.ReLU(inplace=True))
        self.attention = nn.Sequential(nn.Conv2d(128, 64, kernel_size=1), nn.ReLU(inplace=True),
                                       nn.Conv2d(64, 128, kernel_size=1), nn.Sigmoid())
        self.feature_extractor = nn.Sequential(
            nn.Conv2d(128, 256, kernel_size=3, padding=1), nn.BatchNorm2d(256), nn.ReLU(inplace=True),
            nn.AdaptiveAvgPool2d(4),
            nn.Conv2d(256, 512, kernel_size=3, padding=1), nn.BatchNorm2d(512), nn.ReLU(inplace=True))
        self.global_avg_pool = nn.AdaptiveAvgPool2d(1)
        self.fc_layers = nn.Sequential(
            nn.Linear(512, 128), nn.ReLU(inplace=True), nn.Dropout(0.3),
            nn.Linear(128, 64), nn.ReLU(inplace=True), nn.Dropout(0.2),
            nn.Linear(64, 32), nn.ReLU(inplace=True),
            nn.Linear(32, 1))
        self.output_min = 0.01
        self.output_max = 0.5
        self.sigmoid = nn.Sigmoid()
        self.compute_dtype = torch.float32

    def forward(self, depth_image: torch.Tensor) -> torch.Tensor:
        assert depth_image.dim() == 4, f"Expected 4D tensor, got {depth_image.dim()}D"
        assert depth_image.shape[1] == self.input_channels, \
            f"Expected {self.input_channels} channels, got {depth_image.shape[1]}"
        from . import ratio
        return ratio.ratio_predictor_forward(self, depth_image)
