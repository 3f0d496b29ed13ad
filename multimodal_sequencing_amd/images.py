"""Device image pipeline: decoded RGB images -> the model's normalised
[.., 3, 224, 224] f32 input, on the GPU.

The reference transforms every image on the host in its DataLoader (datasets/processors.py:
717-740 -> img_utils.read_and_transform_img_from_filename :135-144 with the transform of
trainers/multimodal_utils.py:195-208: skimage Rescale((224, 224)) + ToTensor + ImageNet
Normalize), then copies float64 images per pair. Here the host only decodes (uint8 HWC, as
skimage.io.imread returns it: grey -> RGB, alpha dropped); the uint8 bytes travel to the device
once and csrc/image.hip resizes (anti-aliased, as skimage 0.17.2 does) and normalises them
straight into the images tensor the pair gather (mmseq_vit_im2col) reads.
"""
import numpy as np
import torch

from . import _native as N

IMAGENET_MEAN = (0.485, 0.456, 0.406)  # trainers/multimodal_utils.py:196-197
IMAGENET_STD = (0.229, 0.224, 0.225)


def as_rgb_uint8(img):
    """img_utils.py:135-142: grey -> RGB (skimage.color.gray2rgb), alpha channel dropped."""
    a = np.asarray(img)
    if a.dtype != np.uint8:
        raise ValueError(f"decoded images are uint8, got {a.dtype}")
    if a.ndim == 2:
        a = np.stack([a, a, a], -1)
    if a.shape[-1] > 3:
        a = a[:, :, :3]
    if a.ndim != 3 or a.shape[-1] != 3:
        raise ValueError(f"image shape {a.shape} is not H x W x 3")
    return np.ascontiguousarray(a)


def decode_image(path):
    """skimage.io.imread equivalent for the formats the datasets hold (PIL decoder)."""
    from PIL import Image
    with Image.open(path) as im:
        return as_rgb_uint8(np.asarray(im))


class DeviceImagePipeline:
    def __init__(self, size=(224, 224), mean=IMAGENET_MEAN, std=IMAGENET_STD, device="cuda"):
        self.size = tuple(size)
        self.mean, self.std = tuple(mean), tuple(std)
        self.device = torch.device(device)

    def __call__(self, images, out=None):
        """images: sequence of uint8 H x W (x 3|4) arrays -> f32 [n][3][oh][ow] on the device
        (written into `out` when given, e.g. a view of the [B][N][3][R][R] batch tensor)."""
        imgs = [as_rgb_uint8(i) for i in images]
        n = len(imgs)
        oh, ow = self.size
        if out is None:
            out = torch.empty(n, 3, oh, ow, dtype=torch.float32, device=self.device)
        if n == 0:
            return out
        hs = [i.shape[0] for i in imgs]
        ws = [i.shape[1] for i in imgs]
        nbytes = [i.size for i in imgs]
        poff = np.concatenate([[0], np.cumsum(nbytes)[:-1]]).astype(np.int64)
        woff = np.concatenate([[0], np.cumsum([h * 3 * ow for h in hs])[:-1]]).astype(np.int64)
        table = np.stack([poff, hs, ws, woff], 1).astype(np.int64)
        host = torch.empty(int(sum(nbytes)), dtype=torch.uint8, pin_memory=True)
        hv = host.numpy()
        for i, o in zip(imgs, poff):
            hv[o:o + i.size] = i.reshape(-1)
        pix = host.to(self.device, non_blocking=True)
        tab = torch.from_numpy(table).pin_memory().to(self.device, non_blocking=True)
        N.image_resize_normalize(pix, tab, hs, max(hs), max(ws), out.view(n, 3, oh, ow),
                                 self.mean, self.std)
        return out

    def stories(self, stories):
        """[B][N] images -> [B][N][3][oh][ow] (the PureClassDataset batch layout,
        processors.py:740-746)."""
        B, Nimg = len(stories), len(stories[0])
        if any(len(s) != Nimg for s in stories):
            raise ValueError("every story needs the same number of images")
        out = torch.empty(B, Nimg, 3, *self.size, dtype=torch.float32, device=self.device)
        self([img for s in stories for img in s], out=out.view(B * Nimg, 3, *self.size))
        return out
