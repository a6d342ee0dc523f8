"""GPU-resident CLIP(+LoRA) encoder: the `model` object load_clip_model returns.

Wraps one libclm context (include/clm.h). Replaces the transformers CLIPModel
(+ peft PeftModel) that models/clip_model.py:59,78 builds: weights are handed
over by their transformers / PEFT state-dict names, LoRA is merged into the
weights (default; zero runtime cost) or kept as a K-extension of the same GEMM
("unmerged", hot-swappable), and every encode runs in hand-written gfx950 HIP
kernels on the caller's current torch stream.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional

import numpy as np
import torch

from . import _capi as C
from .config import ModelConfig

# "mixed": bf16 operands in the vision tower, fp16 in the text tower -- the bf16 assignment that meets
# the path's 1e-3 score bar (the text tower carries the bf16 error: include/clm.h CLM_COMPUTE_MIXED)
_DTYPE_CODES = {"bfloat16": C.CLM_BF16, "bf16": C.CLM_BF16, "float16": C.CLM_F16, "fp16": C.CLM_F16,
                "mixed": C.CLM_COMPUTE_MIXED}
_DTYPE_NAMES = {C.CLM_BF16: "bfloat16", C.CLM_F16: "float16", C.CLM_COMPUTE_MIXED: "mixed"}


class ClipLoraModel:
    def __init__(self, cfg: ModelConfig, device=None, compute_dtype: str = "bfloat16",
                 lora_mode: str = "merged", max_batch: int = 256):
        C.require_gpu()
        L = C.lib()
        self.cfg = cfg
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                   else torch.device(device).index or 0)
        if compute_dtype not in _DTYPE_CODES:
            raise ValueError(f"compute_dtype must be one of {sorted(_DTYPE_CODES)}")
        if lora_mode not in ("merged", "unmerged"):
            raise ValueError("lora_mode must be 'merged' or 'unmerged'")
        self.compute_dtype = _DTYPE_NAMES[_DTYPE_CODES[compute_dtype]]
        self.lora_mode = lora_mode
        self.max_batch = int(max_batch)
        d = C.ModelDesc()
        for tw, src in ((d.vision, cfg.vision), (d.text, cfg.text)):
            tw.hidden, tw.layers, tw.heads, tw.mlp = src.hidden, src.layers, src.heads, src.mlp
        d.patch, d.image_size, d.channels = cfg.patch, cfg.image_size, cfg.channels
        d.vocab, d.max_pos, d.proj_dim = cfg.vocab, cfg.max_pos, cfg.proj_dim
        d.eos_token_id, d.ln_eps = cfg.eos_token_id, cfg.ln_eps
        d.lora_r, d.lora_alpha, d.lora_targets = cfg.lora_r, cfg.lora_alpha, cfg.lora_mask
        d.lora_mode = C.CLM_LORA_MERGED if lora_mode == "merged" else C.CLM_LORA_UNMERGED
        d.compute_dtype = _DTYPE_CODES[compute_dtype]
        d.max_batch = self.max_batch
        for i in range(3):
            d.mean[i], d.std[i] = cfg.mean[i], cfg.std[i]
        self._desc = d
        ctx = ctypes.c_void_p()
        C.check(L.clm_ctx_create(self.device.index, ctypes.byref(d), ctypes.byref(ctx)), "clm_ctx_create")
        self._ctx = ctx
        self.lora_loaded = False
        self.training = False

    # ------------------------------------------------------------ weights --
    def load_tensors(self, tensors: Dict[str, np.ndarray]) -> None:
        L = C.lib()
        for name, arr in tensors.items():
            a = np.ascontiguousarray(np.asarray(arr, dtype=np.float32))
            shape = (ctypes.c_int64 * max(a.ndim, 1))(*a.shape)
            C.check(L.clm_load_tensor(self._ctx, name.encode(), a.ctypes.data_as(ctypes.c_void_p), C.CLM_F32,
                                      shape, a.ndim), f"load {name}")
            if ".lora_A." in name:
                self.lora_loaded = True

    def finalize(self) -> "ClipLoraModel":
        C.check(C.lib().clm_finalize(self._ctx), "clm_finalize")
        return self

    def attach_lora(self, r: int, alpha: float, targets, tensors: Dict[str, np.ndarray]) -> "ClipLoraModel":
        """Attach (or replace) LoRA adapters on THIS model's weights, in place -- what PEFT's
        get_peft_model does to the CLIPModel it is given (models/lora_adapter.py:46-56)."""
        cfg = self.cfg.with_lora(r, alpha, targets)
        C.check(C.lib().clm_set_lora(self._ctx, int(cfg.lora_r), float(cfg.lora_alpha), int(cfg.lora_mask)),
                "clm_set_lora")
        self.cfg = cfg
        self.load_tensors(tensors)
        return self.finalize()

    def set_lora_enabled(self, enabled: bool) -> None:
        C.check(C.lib().clm_set_lora_enabled(self._ctx, int(bool(enabled))), "clm_set_lora_enabled")

    # ------------------------------------------------------------- encode --
    def _out(self, n: int, out_dtype: torch.dtype, out: Optional[torch.Tensor]) -> torch.Tensor:
        if out_dtype not in (torch.float32, torch.float16):
            raise ValueError("out_dtype must be torch.float32 or torch.float16")
        if out is None:
            return torch.empty((n, self.cfg.proj_dim), dtype=out_dtype, device=self.device)
        if out.shape != (n, self.cfg.proj_dim) or out.dtype != out_dtype or not out.is_contiguous():
            raise ValueError("bad `out` tensor")
        return out

    def encode_pixels(self, pixels: torch.Tensor, normalize: bool = True, out_dtype=torch.float32,
                      out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """uint8 [n, S, S, 3] (raw RGB; rescale+normalise fused in-kernel) or float32
        [n, 3, S, S] CLIPProcessor pixel_values -> [n, proj_dim] on the device."""
        S = self.cfg.image_size
        if pixels.dtype == torch.uint8:
            if pixels.dim() != 4 or tuple(pixels.shape[1:]) != (S, S, self.cfg.channels):
                raise ValueError(f"uint8 pixels must be [n, {S}, {S}, {self.cfg.channels}], got {tuple(pixels.shape)}")
            layout = C.CLM_PIX_U8_HWC
        elif pixels.dtype == torch.float32:
            if pixels.dim() != 4 or tuple(pixels.shape[1:]) != (self.cfg.channels, S, S):
                raise ValueError(
                    f"Input image size must be [n, {self.cfg.channels}, {S}, {S}], got {tuple(pixels.shape)}")
            layout = C.CLM_PIX_F32_CHW
        else:
            raise ValueError("pixels must be uint8 NHWC or float32 NCHW")
        pixels = pixels.contiguous()
        n = pixels.shape[0]
        res = self._out(n, out_dtype, out)
        code = C.CLM_F32 if out_dtype == torch.float32 else C.CLM_F16
        C.check(C.lib().clm_encode_image(self._ctx, C.ptr(pixels), layout, n, C.ptr(res), code, int(normalize),
                                         C.stream_of(self.device)), "clm_encode_image")
        return res

    def encode_ids(self, ids: torch.Tensor, normalize: bool = True, out_dtype=torch.float32,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """token ids [n, L] (L <= max_pos, each row containing EOS) -> [n, proj_dim] on the device."""
        if ids.dim() == 1:
            ids = ids.unsqueeze(0)
        if ids.dim() != 2:
            raise ValueError(f"input_ids must be [n, L], got {tuple(ids.shape)}")
        if ids.shape[1] > self.cfg.max_pos:
            raise ValueError(
                f"Sequence length must be less than max_position_embeddings (got `sequence length`: "
                f"{ids.shape[1]} and max_position_embeddings: {self.cfg.max_pos}")
        ids = ids.to(torch.int32).contiguous()
        n, L = ids.shape
        res = self._out(n, out_dtype, out)
        code = C.CLM_F32 if out_dtype == torch.float32 else C.CLM_F16
        C.check(C.lib().clm_encode_text(self._ctx, C.ptr(ids), n, L, C.ptr(res), code, int(normalize),
                                        C.stream_of(self.device)), "clm_encode_text")
        return res

    def encode_pair(self, pixels: torch.Tensor, ids: torch.Tensor, normalize: bool = True,
                    out_dtype=torch.float32, out_img: Optional[torch.Tensor] = None,
                    out_txt: Optional[torch.Tensor] = None, graph: bool = True, split: int = 0):
        """Image batch + caption batch (device tensors, each <= max_batch) encoded concurrently:
        each tower cut into `split` sub-batches (0 = library default), all pieces on their own
        streams; graph=True replays a captured hipGraph for repeated identical calls."""
        if not 0 <= int(split) <= 15:
            raise ValueError("split must be in [0, 15]")
        S = self.cfg.image_size
        if pixels.dtype == torch.uint8 and tuple(pixels.shape[1:]) == (S, S, self.cfg.channels):
            layout = C.CLM_PIX_U8_HWC
        elif pixels.dtype == torch.float32 and tuple(pixels.shape[1:]) == (self.cfg.channels, S, S):
            layout = C.CLM_PIX_F32_CHW
        else:
            raise ValueError("pixels must be uint8 NHWC or float32 NCHW of the model's image size")
        if ids.dim() != 2 or ids.dtype != torch.int32:
            raise ValueError("ids must be int32 [n, L]")
        if not (pixels.is_cuda and ids.is_cuda):
            raise ValueError("encode_pair needs device tensors")
        pixels, ids = pixels.contiguous(), ids.contiguous()
        oi = self._out(pixels.shape[0], out_dtype, out_img)
        ot = self._out(ids.shape[0], out_dtype, out_txt)
        code = C.CLM_F32 if out_dtype == torch.float32 else C.CLM_F16
        C.check(C.lib().clm_encode_pair(self._ctx, C.ptr(pixels), layout, pixels.shape[0], C.ptr(ids),
                                        ids.shape[0], ids.shape[1], C.ptr(oi), C.ptr(ot), code, int(normalize),
                                        (C.CLM_PAIR_GRAPH if graph else 0) | (int(split) << C.CLM_PAIR_SPLIT_SHIFT),
                                        C.stream_of(self.device)),
                "clm_encode_pair")
        return oi, ot

    def pair_path(self) -> str:
        """how the last encode_pair ran: "streams" (a stream per tower piece) or "none" (no call yet)"""
        return {0: "streams"}.get(C.lib().clm_pair_path(self._ctx), "none")

    # ------------------------------------------------------------ timing --
    def prof_enable(self, enable: bool = True) -> None:
        C.check(C.lib().clm_prof_enable(self._ctx, int(bool(enable))), "clm_prof_enable")

    def prof_read(self) -> dict:
        """{category: (kernel_ms, algorithmic_work, launches)} since prof_enable (HIP events on the
        launch stream); work is FLOPs for gemm/attn, bytes for ln/other."""
        out = {}
        for name, cat in (("gemm", C.CLM_PROF_GEMM), ("attn", C.CLM_PROF_ATTN), ("ln", C.CLM_PROF_LN),
                          ("other", C.CLM_PROF_OTHER)):
            ms, work, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
            C.check(C.lib().clm_prof_read(self._ctx, cat, ctypes.byref(ms), ctypes.byref(work), ctypes.byref(n)),
                    "clm_prof_read")
            out[name] = (ms.value, work.value, n.value)
        return out

    # transformers-style entry points (un-normalised projections, like CLIPModel.get_*_features
    # .pooler_output; TF/models/clip/modeling_clip.py:683-754)
    def get_image_features(self, pixel_values: torch.Tensor) -> torch.Tensor:
        return self.encode_pixels(pixel_values, normalize=False)

    def get_text_features(self, input_ids: torch.Tensor, attention_mask=None) -> torch.Tensor:
        # attention_mask only marks pads after EOS; the causal mask already hides them from the
        # pooled EOS row, so it does not change the result
        return self.encode_ids(input_ids, normalize=False)

    # nn.Module-like conveniences the reference calls (clip_model.py:81,111; embed_image.py:35)
    def eval(self) -> "ClipLoraModel":
        return self

    def to(self, *args, **kwargs) -> "ClipLoraModel":
        return self

    def parameters(self):
        yield torch.empty(0, dtype=torch.float32, device=self.device)

    def close(self) -> None:
        if getattr(self, "_ctx", None):
            try:
                C.lib().clm_ctx_destroy(self._ctx)
            finally:
                self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
