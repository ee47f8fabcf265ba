"""``yolov8.tools``: ``loss`` here is the fused GPU ComputeLoss (tools/loss.py:94-677 interface) and
``simplified_loss`` the ``SimplifiedYOLOLoss`` drop-in train.py imports (train.py:14,321-330; ComputeLoss
semantics, see its docstring); both always shadow the reference's modules of the same name.  The reference's other tools (dataset,
training loop, utils: outside the hot path) resolve from the reference checkout when
``YMS_REFERENCE_ROOT`` is set; the input pipeline's GPU half is ``yms.data``."""
import os as _os

_ref = _os.environ.get("YMS_REFERENCE_ROOT")
if _ref:
    __path__.append(_os.path.join(_ref, "yolov8", "tools"))
