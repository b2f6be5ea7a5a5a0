"""Object-detection model family (Mask R-CNN, SSD-ResNet34, Faster/Mask
R-CNN and RetinaNet inference, SSD-MobileNet, YOLOv4) built on the HIP detection ops
(bitmask NMS, ROIAlign, sigmoid focal loss) and the NHWC bf16 ResNet bodies."""
from .box_ops import AnchorGenerator, BoxCoder, Matcher, box_iou  # noqa: F401
from .backbone import FPN, ResNetFPN, freeze_bn  # noqa: F401
from .rcnn import (GeneralizedRCNN, faster_rcnn_resnet50_fpn, mask_rcnn_resnet50_fpn,  # noqa: F401
                   mask_rcnn_resnext101_32x8d_fpn, synthetic_detection_batch)
from .roi_heads import paste_masks  # noqa: F401
