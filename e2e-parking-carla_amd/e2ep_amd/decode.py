"""GPU frame decode over csrc/decode.hip: cached uint8 crops -> the reference's tensors.

decode_frames: (F, H, W, 3) uint8 camera / CARLA-depth crops (optionally gathered through a
source-frame table) -> image (F, 3, H, W) fp32 normalised exactly as torchvision
ToTensor + Normalize, depth (F, H, W) float64 metres exactly as get_depth
(dataset/carla_dataset.py:114-131, :494-515).  widen_rows: uint8 class maps -> int64."""
import torch

from . import _lib


def _check(t, name, dtype):
    if not t.is_cuda:
        raise _lib.E2EPError(f"decode: {name} must be on the HIP device")
    if t.dtype != dtype or not t.is_contiguous():
        raise _lib.E2EPError(f"decode: {name} must be contiguous {dtype}, got {t.dtype}")


def _index(src, n_src, device, what):
    """Bounds-check a gather table on the host (a bad index would fault the kernel), then
    move it to the device."""
    if src is None:
        return None
    src = torch.as_tensor(src, dtype=torch.int64)
    if src.is_cuda:
        raise _lib.E2EPError(f"{what}: pass the source index as a host tensor (it is "
                             "bounds-checked before the launch)")
    src = src.reshape(-1)
    if src.numel() and (int(src.min()) < 0 or int(src.max()) >= n_src):
        raise _lib.E2EPError(f"{what}: source index outside [0, {n_src})")
    return src.to(device=device, non_blocking=True)


def decode_frames(rgb=None, depth_rgb=None, src_frame=None, out_image=None, out_depth=None):
    """rgb / depth_rgb: (S, H, W, 3) uint8 on the device (either may be None).  Output frame
    f reads source frame src_frame[f] (a host int64 tensor; all S frames in order when None).  Returns
    (image (F, 3, H, W) fp32 or None, depth (F, H, W) fp64 or None)."""
    ref = rgb if rgb is not None else depth_rgb
    if ref is None:
        return None, None
    for t, n in ((rgb, "rgb"), (depth_rgb, "depth_rgb")):
        if t is not None:
            _check(t, n, torch.uint8)
            if t.dim() != 4 or t.shape[-1] != 3 or t.shape[1:] != ref.shape[1:]:
                raise _lib.E2EPError(f"decode: {n} must be (S, H, W, 3), got {tuple(t.shape)}")
    S, H, W = ref.shape[:3]
    if rgb is not None and depth_rgb is not None and rgb.shape[0] != depth_rgb.shape[0]:
        raise _lib.E2EPError("decode: rgb and depth_rgb hold different frame counts")
    idx = _index(src_frame, S, ref.device, "decode")
    F = S if idx is None else idx.numel()
    image = depth = None
    if rgb is not None:
        image = out_image if out_image is not None else torch.empty(F, 3, H, W, device=ref.device)
        _check(image, "out_image", torch.float32)
        if image.shape != (F, 3, H, W):
            raise _lib.E2EPError(f"decode: out_image {tuple(image.shape)} != {(F, 3, H, W)}")
    if depth_rgb is not None:
        depth = out_depth if out_depth is not None else torch.empty(
            F, H, W, dtype=torch.float64, device=ref.device)
        _check(depth, "out_depth", torch.float64)
        if depth.shape != (F, H, W):
            raise _lib.E2EPError(f"decode: out_depth {tuple(depth.shape)} != {(F, H, W)}")
    _lib.call("e2ep_decode_frames", _lib.ptr(rgb), _lib.ptr(depth_rgb), _lib.ptr(idx), F, H * W,
              _lib.ptr(image), _lib.ptr(depth), _lib.stream())
    return image, depth


def widen_rows(src, src_row=None, out=None):
    """(S, ...) uint8 rows -> (R, ...) int64, row r = src[src_row[r]] (all rows when None)."""
    _check(src, "src", torch.uint8)
    S = src.shape[0]
    row_len = src[0].numel() if S else 0
    idx = _index(src_row, S, src.device, "widen_rows")
    R = S if idx is None else idx.numel()
    dst = out if out is not None else torch.empty((R,) + tuple(src.shape[1:]), dtype=torch.int64,
                                                  device=src.device)
    _check(dst, "out", torch.int64)
    if dst.numel() != R * row_len:
        raise _lib.E2EPError(f"widen_rows: out holds {dst.numel()} elements, need {R * row_len}")
    if R and row_len:
        _lib.call("e2ep_widen_u8_i64", _lib.ptr(src), _lib.ptr(idx), R, row_len, _lib.ptr(dst),
                  _lib.stream())
    return dst
