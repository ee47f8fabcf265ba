"""The reference's tools/ (dataset, training loop, loss, utils) are outside the hot path;
with ``YMS_REFERENCE_ROOT`` set they resolve from the reference checkout."""
import os as _os

_ref = _os.environ.get("YMS_REFERENCE_ROOT")
if _ref:
    __path__.append(_os.path.join(_ref, "yolov8", "tools"))
