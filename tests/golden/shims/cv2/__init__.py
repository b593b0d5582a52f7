"""Stand-in for the two OpenCV calls metrics/calculate_ssim.py makes (cv2 is not
installed in the build container). Test infrastructure only, used by
tests/golden/make_golden.py when it imports the reference's SSIM to write fixtures.

getGaussianKernel(ksize, sigma): OpenCV's documented sampled Gaussian for sigma > 0,
G_i = exp(-(i - (ksize-1)/2)^2 / (2 sigma^2)) normalised to sum 1, float64, shape (ksize, 1).
filter2D(src, -1, kernel): correlation (not convolution) with the anchor at the kernel
centre and BORDER_REFLECT_101 (scipy 'mirror'); the reference crops [5:-5, 5:-5], so the
border rule never reaches its result.
"""
import numpy as np
from scipy import ndimage


def getGaussianKernel(ksize, sigma):
    x = np.arange(ksize, dtype=np.float64) - (ksize - 1) * 0.5
    g = np.exp((-0.5 / (sigma * sigma)) * x * x)
    return (g / g.sum()).reshape(ksize, 1)


def filter2D(src, ddepth, kernel):
    return ndimage.correlate(np.asarray(src, dtype=np.float64), np.asarray(kernel, dtype=np.float64), mode='mirror')
