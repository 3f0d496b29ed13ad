"""CPU float64 restatement of the reference's image transform — TEST INFRASTRUCTURE ONLY (used by
tests/ as the checker of csrc/image.hip; never imported by the product package).

Reference path: trainers/multimodal_utils.py:195-208 builds
    Compose([Rescale((224, 224)), ToTensor(), Normalize(ImageNet mean, std)])
and datasets/img_utils.py applies it to skimage.io.imread output (:135-144: grey -> RGB, alpha
dropped). Rescale (:27-56) calls skimage.transform.resize(image, (224, 224)) with its defaults.

skimage is a third-party dependency absent from this image: scikit-image 0.17.2 and scipy 1.5.3
are pinned by the reference (requirements.txt:256, 258). Its published resize algorithm is
restated here with scipy.ndimage (present):
  1. image -> float64 in [0, 1] (img_as_float: uint8 / 255);
  2. anti_aliasing (default True when resizing): ndimage.gaussian_filter with per-axis sigma
     max(0, (in / out - 1) / 2) (channel axis 0), mode 'mirror' (skimage 'reflect'),
     truncate 4.0;
  3. warp with the affine map out -> in: r = in / out * (o + 0.5) - 0.5 per axis (pixel centres
     aligned), order 1 (bilinear), mode 'reflect' (numpy-pad reflect = ndimage 'mirror');
  4. clip to the filtered image's [min, max] (a no-op for bilinear);
then ToTensor (HWC -> CHW, img_utils.py:88-100) and Normalize ((x - mean) / std).
No reference output of this transform exists in /root/reference (no images are shipped), so
this oracle's parity is UNPINNED against the reference itself.
"""
import numpy as np
from scipy import ndimage as ndi

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def skimage_resize(img_u8, out_h, out_w):
    img = np.asarray(img_u8, dtype=np.float64) / 255.0
    H, W, C = img.shape
    factors = np.array([H / out_h, W / out_w, 1.0])
    sigma = np.maximum(0.0, (factors - 1.0) / 2.0)
    filt = ndi.gaussian_filter(img, sigma, mode="mirror", cval=0.0, truncate=4.0)
    rr = factors[0] * (np.arange(out_h) + 0.5) - 0.5
    cc = factors[1] * (np.arange(out_w) + 0.5) - 0.5
    gr, gc = np.meshgrid(rr, cc, indexing="ij")
    out = np.stack([ndi.map_coordinates(filt[..., c], [gr, gc], order=1, mode="mirror")
                    for c in range(C)], -1)
    return np.clip(out, filt.min(), filt.max())


def transform(img_u8, size=(224, 224), mean=IMAGENET_MEAN, std=IMAGENET_STD):
    """uint8 H x W x 3 -> float64 [3][size] as the reference's img_transform_func returns it."""
    a = np.asarray(img_u8)
    if a.ndim == 2:
        a = np.stack([a, a, a], -1)
    a = a[:, :, :3]
    x = skimage_resize(a, *size).transpose(2, 0, 1)
    return (x - np.asarray(mean)[:, None, None]) / np.asarray(std)[:, None, None]
