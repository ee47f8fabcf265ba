"""MI355X-native drop-in for the reference's `yolov8` package (YOLOv8 / YOLO-MS detector).

Only the hot path lives here (model/, yolov8.py).  Set ``YMS_REFERENCE_ROOT`` to an
existing checkout of the reference to let its out-of-scope modules (tools.dataset,
tools.utils, tools.loss, ...) resolve from there: ``from yolov8.tools.dataset import
COCODataset`` then keeps working while ``from yolov8.yolov8 import YOLOv8`` gets this
package.  See INTEGRATION.md."""
import os as _os

_ref = _os.environ.get("YMS_REFERENCE_ROOT")
if _ref:
    __path__.append(_os.path.join(_ref, "yolov8"))
