"""Reference ``operators`` package on the HIP path: iou_utils, Loss, Deformable_convolution."""
