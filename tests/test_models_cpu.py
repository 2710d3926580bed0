"""CPU tests of the model definitions, BN folding, preprocessing and the CLI."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F
from PIL import Image, ImageOps

from semantic_segmentation_server_amd import config as C
from semantic_segmentation_server_amd.labels import load_labels, parse_labels, pascal_colormap
from semantic_segmentation_server_amd.models.deeplab import build_model, count_macs
from semantic_segmentation_server_amd.models.layers import ConvBNAct
from semantic_segmentation_server_amd.models.mobilenetv2 import mnv2_block_specs
from semantic_segmentation_server_amd.ops import reference_ops as R


def test_mac_counts_match_survey():
    assert count_macs(build_model("mnv2", calibrate_hw=None), 513, 513) == pytest.approx(5.3635e9, rel=1e-3)
    assert count_macs(build_model("mnv2", aspp="mobile", calibrate_hw=None), 513, 513) == \
        pytest.approx(2.7407e9, rel=1e-3)


def test_output_stride_16_dilation_schedule():
    stem, specs = mnv2_block_specs(1.0, 16)
    assert stem == 32 and len(specs) == 17
    strides = [s.stride for s in specs]
    dils = [s.dilation for s in specs]
    assert strides == [1, 2, 1, 2, 1, 1, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1]
    assert dils[-4:] == [1, 2, 2, 2]   # 160-stage: first unit rate 1, then 2 (TF-slim)
    m = build_model("mnv2", calibrate_hw=None)
    assert m(torch.zeros(1, 3, 513, 513)).shape == (1, 21, 33, 33)


def test_bn_fold_equivalence():
    torch.manual_seed(0)
    layer = ConvBNAct(16, 24, 3, 2, 2, act=None)
    layer.bn.running_mean.normal_()
    layer.bn.running_var.uniform_(0.5, 2)
    layer.bn.weight.data.normal_()
    layer.eval()
    x = torch.randn(2, 16, 19, 19)
    w, b = layer.fold()
    ref = layer(x)
    got = F.conv2d(x, w, b, 2, 2, 2)
    assert torch.allclose(ref, got, atol=1e-5)


def test_random_init_is_deterministic():
    a = build_model("mnv2", seed=3, calibrate_hw=33)
    b = build_model("mnv2", seed=3, calibrate_hw=33)
    for (ka, va), (kb, vb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert torch.equal(va, vb), ka


def test_pil_nearest_lut_bitexact():
    rng = np.random.default_rng(0)
    for _ in range(20):
        n_in, n_out = int(rng.integers(2, 1500)), int(rng.integers(2, 1100))
        a = np.zeros((1, n_in, 3), np.uint8)
        a[0, :, 0] = np.arange(n_in) % 256
        a[0, :, 1] = np.arange(n_in) // 256
        r = np.asarray(Image.fromarray(a).resize((n_out, 1), Image.NEAREST)).astype(np.int64)
        assert np.array_equal(r[0, :, 0] + 256 * r[0, :, 1], R.pil_nearest_index(n_in, n_out))


@pytest.mark.parametrize("cam", [(640, 480), (1280, 720), (480, 640), (300, 200)])
def test_preprocess_matches_pil_letterbox(cam):
    cw, ch = cam
    rng = np.random.default_rng(1)
    f = rng.integers(0, 256, (ch, cw, 3), dtype=np.uint8)
    lx, ly, rw, rh, _, _ = R.letterbox_luts(cw, ch, 513, 513)
    pil = Image.fromarray(f[..., ::-1].copy()).resize((rw, rh), Image.NEAREST)
    pil = ImageOps.expand(pil, (0, 0, 513 - rw, 513 - rh))
    ref = np.asarray(pil).astype(np.float32) / 127.5 - 1
    out = R.preprocess(torch.from_numpy(f[None]), lx, ly)[0].permute(1, 2, 0).numpy()
    assert np.abs(out - ref).max() < 1e-6


def test_labels_and_colormap():
    lab = load_labels()
    assert lab[0] == "background" and lab[15] == "person" and lab[255] == "ignore" and len(lab) == 22
    assert parse_labels("0 a\n\n1  b c \n") == {0: "a", 1: "b c"}
    # reference algorithm, written independently
    cmap = np.zeros((256, 3), int)
    ind = np.arange(256)
    for shift in range(7, -1, -1):
        for ch in range(3):
            cmap[:, ch] |= ((ind >> ch) & 1) << shift
        ind >>= 3
    assert np.array_equal(cmap, pascal_colormap())


def test_cli_reference_flags_and_defaults():
    cfg = C.parse([])
    assert (cfg.camera_idx, cfg.num_detections, cfg.min_area_ratio, cfg.keep_aspect_ratio) == (1, 3, 0.05, True)
    assert cfg.port == 50051 and cfg.max_workers == 10
    cfg = C.parse(["--no_keep_aspect_ratio", "--num_detections", "5", "--buffer_max", "0"])
    assert cfg.keep_aspect_ratio is False and cfg.num_detections == 5 and cfg.buffer_max is None
    assert C.parse(["--keep_aspect_ratio"]).keep_aspect_ratio is True
    assert C.parse(["--dataset", "cityscapes"]).labels.endswith("cityscapes_labels.txt")
