"""libwdr's own readers of the VAD / diarization model files -- the
whisper.cpp Silero ggml file and the two ONNX graphs (hand-written protobuf subset +
structural mapping, csrc/model_files.cpp) -- checked on the host (no GPU) through the
wdr_dbg_model_file seam: every tensor the loader maps must equal, bit for bit, the oracle
weight the test wrote into the file (tests/model_writers.py).  Reference load sites:
src/vad.rs:18 (WhisperVadContext::new), src/engine.rs:90-91,117 and src/transcribe.rs:343,466
(pyannote-rs -> ONNX Runtime sessions).  Parity with the real downloaded files is unpinned
(none exist offline); the layouts are restated from the published converters / exporters."""
import numpy as np
import pytest

import wdr
from tests.model_writers import write_campplus_onnx, write_segmentation_onnx, write_silero_ggml


def _same(got, want):
    assert sorted(got) == sorted(want), set(got) ^ set(want)
    for k in want:
        np.testing.assert_array_equal(got[k], np.asarray(want[k], np.float32).reshape(-1), err_msg=k)


@pytest.mark.parametrize("ftype16", [True, False])
def test_silero_ggml_tensors(tmp_path, ftype16):
    p = str(tmp_path / "ggml-silero-v5.1.2.bin")
    W = write_silero_ggml(p, ftype16=ftype16)
    got = wdr.model_file_tensors("silero", p)
    _same(got, {k: W[k].astype(np.float16 if ftype16 or k == "stft" else W[k].dtype).astype(np.float32)
                 if W[k].ndim > 1 or k == "stft" else W[k] for k in W})


@pytest.mark.parametrize("gemm", [False, True])
def test_segmentation_onnx_tensors(tmp_path, gemm):
    p = str(tmp_path / "segmentation-3.0.onnx")
    W = write_segmentation_onnx(p, gemm=gemm)
    got = wdr.model_file_tensors("segmentation", p)
    want = dict(W)
    want.pop("sinc.bias", None)
    _same(got, want)


@pytest.mark.parametrize("fused", [False, True])
def test_campplus_onnx_tensors(tmp_path, fused):
    p = str(tmp_path / "cam.onnx")
    W = write_campplus_onnx(p, fused=fused)
    _same(wdr.model_file_tensors("campplus", p), W)


def test_model_file_errors(tmp_path):
    seg = str(tmp_path / "seg.onnx")
    write_segmentation_onnx(seg)
    with pytest.raises(wdr.WdrError, match="embedding model"):
        wdr.model_file_tensors("campplus", seg)       # a segmentation graph is not CAM++
    data = open(seg, "rb").read()
    cut = str(tmp_path / "cut.onnx")
    open(cut, "wb").write(data[:len(data) // 2])
    with pytest.raises(wdr.WdrError, match="failed to load"):
        wdr.model_file_tensors("segmentation", cut)
    vad = str(tmp_path / "vad.bin")
    write_silero_ggml(vad)
    with pytest.raises(wdr.WdrError, match="Silero VAD model"):
        wdr.model_file_tensors("silero", seg)
    with pytest.raises(wdr.WdrError, match="doesn't exist"):
        wdr.model_file_tensors("silero", str(tmp_path / "none.bin"))


def test_campplus_onnx_conditioned_weights_exact(tmp_path):
    """The diarized fixtures' speaker-conditioned CAM++ (tests/golden/make_cam_conditioning.py)
    written as an ONNX file: the loader must reproduce the oracle's weights bit for bit (BN as
    scale / shift with mean 0, var 1, epsilon 0; the conditioned dense layer with its bias)."""
    import os
    from oracle.diarize import cam_weights_conditioned
    W = cam_weights_conditioned(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                             "cam_conditioning.npz"))
    p = str(tmp_path / "cam_cond.onnx")
    out = write_campplus_onnx(p, weights=W)
    _same(wdr.model_file_tensors("campplus", p), out)
    for k in W:
        np.testing.assert_array_equal(out[k], W[k], err_msg=k)
