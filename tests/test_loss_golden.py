"""Pin the loss restatement (oracle/loss_ref.py) against fixtures produced by the REFERENCE's own
``ComputeLoss`` (yolov8/tools/loss.py:94-677, run in the build container by
tests/golden/make_loss_golden.py).  Cases: every IoU variant, an image without GT, a GT with no
foreground, two classes sharing anchors, BCE pos_weight, bf16-rounded maps, the 640 grid at nc = 80.
CPU-only: runs in the "not gpu" tier."""
import numpy as np
import pytest
import torch

import vectors as V
from oracle import loss_ref as R

CASES = ["small", "nogt", "posw", "bf16", "g640"]


def oracle_on_case(z, iou, dtype=torch.float32):
    preds = [torch.from_numpy(m.copy()).to(dtype).requires_grad_(True) for m in z["maps"]]
    pw = None if "pos_weight" not in z else torch.from_numpy(z["pos_weight"]).to(dtype)
    total, items = R.compute_loss(preds, torch.from_numpy(z["targets"]).to(dtype), z["nc"], z["img"],
                                  iou_type=iou, pos_weight=pw)
    total.backward()
    vals = np.array([total.item(), items["loss_box"].item(), items["loss_cls"].item(),
                     items["loss_dfl"].item()])
    return vals, [p.grad.double().numpy() for p in preds]


def grad_rows(z, grads):
    """[B*A, 64 + nc] rows in the fixture's flattening (levels concatenated per image)."""
    B, C = z["B"], 64 + z["nc"]
    return np.concatenate([g.reshape(B, C, -1).transpose(0, 2, 1) for g in grads], 1).reshape(-1, C)


def check_against_fixture(z, iou, vals, grads, vtol, gtol):
    ref = z[f"{iou}:loss"].astype(np.float64)
    err = np.abs(vals - ref) / np.maximum(np.abs(ref), 1e-3)
    assert err.max() <= vtol, (iou, vals.tolist(), ref.tolist())
    if f"{iou}:grad0" in z:
        for i, g in enumerate(grads):
            r = z[f"{iou}:grad{i}"].astype(np.float64)
            rel = np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-30)
            assert rel <= gtol, (iou, i, rel)
        return
    rows = grad_rows(z, grads)
    fg = z[f"{iou}:fg_rows"]
    mine_fg = np.nonzero(np.any(rows[:, :64] != 0, axis=1))[0]
    assert np.array_equal(mine_fg, fg), "foreground anchors differ from the reference's"
    for key in ("fg", "samp"):
        r = z[f"{iou}:{key}_grad"].astype(np.float64)
        g = rows[z[f"{iou}:{key}_rows"]]
        rel = np.linalg.norm(g - r) / max(np.linalg.norm(r), 1e-30)
        assert rel <= gtol, (iou, key, rel)
    for i, g in enumerate(grads):
        g64 = g.ravel()
        w = V.checksum_weights(g64.size, 7 + i)
        ck = np.array([g64 @ w, np.abs(g64).sum(), np.sqrt(g64 @ g64)])
        ref = z[f"{iou}:cksum{i}"]
        assert np.all(np.abs(ck - ref) <= gtol * np.abs(ref[1:2]) + 1e-12), (iou, i, ck.tolist(), ref.tolist())


@pytest.mark.parametrize("name", CASES)
def test_loss_oracle_matches_reference_fixtures(name):
    """fp32 restatement vs the reference in fp32: the same ops in the same order, so the loss terms
    and every gradient element are bit-identical."""
    z = V.load_loss_case(name)
    for iou in z["ious"]:
        vals, grads = oracle_on_case(z, iou)
        vals = vals.astype(np.float32).astype(np.float64)
        check_against_fixture(z, iou, vals, grads, vtol=0.0, gtol=0.0)


def test_loss_fixtures_cover_the_edge_cases():
    small = V.load_loss_case("small")
    assert small["ious"] == ["ciou", "diou", "giou", "iou"]
    tg = small["targets"]
    assert not np.any(tg[:, 0] == 1) or np.all(tg[tg[:, 0] == 1, 4] < 0.01)   # image 1: only the tiny GT
    nogt = V.load_loss_case("nogt")
    assert nogt["targets"].shape == (0, 6) and nogt["ciou:loss"][1] == 0 and nogt["ciou:loss"][3] == 0
    g640 = V.load_loss_case("g640")
    assert g640["nc"] == 80 and sum(h * w for h, w in g640["shapes"]) == 8400
    assert len(g640["ciou:fg_rows"]) > 50 and g640["ciou:loss"][1] > 0
    assert "pos_weight" in V.load_loss_case("posw")
