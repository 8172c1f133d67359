"""Test infrastructure: write the VAD / diarization model files the reference downloads
 from the oracle's weights, so libwdr's loaders can be checked without
any real model (none exist offline):

* whisper.cpp's Silero VAD file (`ggml-silero-v5.1.2.bin` layout, see
  csrc/model_files.cpp load_silero_ggml);
* `segmentation-3.0.onnx` and `wespeaker_en_voxceleb_CAM++.onnx` as ONNX ModelProtos, hand-
  encoded protobuf (no `onnx` package here), with the node structure torch.onnx.export gives
  these modules: InstanceNormalization / Conv / LSTM (ONNX gate order i, o, f, c) / MatMul + Add
  or Gemm for PyanNet; Conv / BatchNormalization (separate, or fused into the conv's bias the way
  the exporter's eval-mode Conv+BN fusion leaves it) / Relu / Add / Concat / ... for CAM++.

Each writer returns the oracle weight dict the file encodes, so tests compare the GPU against
the oracle on exactly the file's numbers.
"""
import struct

import numpy as np

# ---------------------------------------------------------------- protobuf encoding


def _varint(v):
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field, wt):
    return _varint((field << 3) | wt)


def _len(field, payload):
    return _key(field, 2) + _varint(len(payload)) + payload


def _str(field, s):
    return _len(field, s.encode())


def _int(field, v):
    return _key(field, 0) + _varint(v)


def tensor_proto(name, arr, dtype="f32"):
    a = np.asarray(arr)
    body = _len(1, b"".join(_varint(int(d)) for d in a.shape))   # dims, packed
    if dtype == "f16":
        body += _int(2, 10) + _str(8, name) + _len(9, np.ascontiguousarray(a, "<f2").tobytes())
    elif dtype == "i64":
        body += _int(2, 7) + _str(8, name) + _len(9, np.ascontiguousarray(a, "<i8").tobytes())
    elif dtype == "f32_float_data":   # the float_data field instead of raw_data
        body += _int(2, 1) + _str(8, name) + _len(4, np.ascontiguousarray(a, "<f4").tobytes())
    else:
        body += _int(2, 1) + _str(8, name) + _len(9, np.ascontiguousarray(a, "<f4").tobytes())
    return body


def _attr(name, v):
    body = _str(1, name)
    if isinstance(v, float):
        body += _key(2, 5) + struct.pack("<f", v) + _int(20, 1)
    elif isinstance(v, int):
        body += _int(3, v) + _int(20, 2)
    elif isinstance(v, str):
        body += _len(4, v.encode()) + _int(20, 3)
    elif isinstance(v, (list, tuple)):
        body += _len(8, b"".join(_varint(int(x)) for x in v)) + _int(20, 7)
    else:
        raise TypeError(v)
    return body


class Graph:
    def __init__(self):
        self.nodes, self.inits, self.n = [], [], 0

    def tmp(self):
        self.n += 1
        return "t%d" % self.n

    def init(self, arr, dtype="f32", name=None):
        name = name or "onnx::w%d" % (len(self.inits) + 1)
        self.inits.append(tensor_proto(name, arr, dtype))
        return name

    def node(self, op, inputs, n_out=1, **attrs):
        outs = [self.tmp() for _ in range(n_out)]
        body = b"".join(_str(1, i) for i in inputs) + b"".join(_str(2, o) for o in outs)
        body += _str(3, "%s_%d" % (op, len(self.nodes))) + _str(4, op)
        body += b"".join(_len(5, _attr(k, v)) for k, v in attrs.items())
        self.nodes.append(body)
        return outs[0] if n_out == 1 else outs

    def model(self, inp, out):
        vi = lambda n: _str(1, n)   # ValueInfoProto: name only
        g = b"".join(_len(1, n) for n in self.nodes) + _str(2, "main_graph")
        g += b"".join(_len(5, t) for t in self.inits) + _len(11, vi(inp)) + _len(12, vi(out))
        opset = _str(1, "") + _int(2, 17)
        return _int(1, 8) + _str(2, "pytorch") + _str(3, "2.1.0") + _len(7, g) + _len(8, opset)


# ---------------------------------------------------------------- segmentation-3.0


def _mutate(W, seed, keys=None):
    """Scale every tensor by a seeded factor in [0.8, 1.2] (and shift biases) so that a loader
    which ignored the file (synthetic weights) could not match."""
    rng = np.random.default_rng(seed)
    for k in sorted(W):
        if keys is not None and k not in keys:
            continue
        W[k] = (W[k] * np.float32(rng.uniform(0.8, 1.2))).astype(W[k].dtype)
    return W


def write_segmentation_onnx(path, seed=1, gemm=False):
    """PyanNet (segmentation-3.0) with the oracle's seg_weights(), mutated (seed None: as
    they are).  gemm: linear layers as Gemm(transB=1) instead of MatMul + Add."""
    from oracle import diarize as D
    W = D.seg_weights() if seed is None else _mutate(D.seg_weights(), seed)
    g = Graph()
    x = "input_values"
    x = g.node("InstanceNormalization", [x, g.init(W["wav_norm.weight"]), g.init(W["wav_norm.bias"])], epsilon=1e-5)
    x = g.node("Conv", [x, g.init(W["sinc.weight"])], strides=[10], kernel_shape=[251])
    x = g.node("Abs", [x])
    for i, (cw, cb) in enumerate([(None, None), ("conv1.weight", "conv1.bias"), ("conv2.weight", "conv2.bias")]):
        if cw is not None:
            x = g.node("Conv", [x, g.init(W[cw]), g.init(W[cb])], kernel_shape=[5])
        x = g.node("MaxPool", [x], kernel_shape=[3], strides=[3])
        x = g.node("InstanceNormalization", [x, g.init(W["norm%d.weight" % i]), g.init(W["norm%d.bias" % i])],
                   epsilon=1e-5)
        x = g.node("LeakyRelu", [x], alpha=0.01)
    x = g.node("Transpose", [x], perm=[2, 0, 1])
    torch_to_onnx = [0, 3, 1, 2]   # ONNX block j <- torch block (i, o, f, c from i, f, g, o)
    for l in range(4):
        Ws, Rs, Bs = [], [], []
        for d in ("", "_reverse"):
            wih, whh = W["lstm.weight_ih_l%d%s" % (l, d)], W["lstm.weight_hh_l%d%s" % (l, d)]
            bih, bhh = W["lstm.bias_ih_l%d%s" % (l, d)], W["lstm.bias_hh_l%d%s" % (l, d)]
            blk = lambda a: np.concatenate([a[j * 128:(j + 1) * 128] for j in torch_to_onnx], 0)
            Ws.append(blk(wih))
            Rs.append(blk(whh))
            Bs.append(np.concatenate([blk(bih), blk(bhh)]))
        y = g.node("LSTM", [x, g.init(np.stack(Ws)), g.init(np.stack(Rs)), g.init(np.stack(Bs)), ""], n_out=3,
                   direction="bidirectional", hidden_size=128)[0]
        y = g.node("Transpose", [y], perm=[0, 2, 1, 3])
        x = g.node("Reshape", [y, g.init(np.array([0, 0, -1]), "i64")])
    x = g.node("Transpose", [x], perm=[1, 0, 2])
    for name, act in (("linear0", True), ("linear1", True), ("classifier", False)):
        if gemm:
            x = g.node("Gemm", [x, g.init(W[name + ".weight"]), g.init(W[name + ".bias"])], transB=1)
        else:
            x = g.node("MatMul", [x, g.init(np.ascontiguousarray(W[name + ".weight"].T))])
            x = g.node("Add", [g.init(W[name + ".bias"]), x])
        if act:
            x = g.node("LeakyRelu", [x], alpha=0.01)
    out = g.node("LogSoftmax", [x], axis=-1)
    with open(path, "wb") as f:
        f.write(g.model("input_values", out))
    return W


# ---------------------------------------------------------------- CAM++


def write_campplus_onnx(path, seed=2, fused=False, weights=None):
    """wespeaker CAMPPlus with the oracle's cam_weights().  Unfused: every BN a
    BatchNormalization node with seeded (gamma, beta, mean, var); fused: the conv+BN pairs
    become one Conv with a bias (the exporter's eval-mode fusion), standalone BNs stay.
    weights (an oracle dict, e.g. oracle/diarize.py cam_weights_conditioned()): written exactly --
    every BN as (gamma, beta) = (scale, shift) with mean 0, var 1, epsilon 0 (folded bit-exact by
    the loader), the dense layer as a Conv with its bias (its BN scale must be 1).
    Returns the oracle dict of the effective weights (BN folded in double, as the loader)."""
    from oracle import diarize as D
    exact = weights is not None
    W = weights if exact else D.cam_weights()
    rng = np.random.default_rng(seed)
    eps = np.float32(0.0 if exact else 1e-5)
    g = Graph()
    out_W = {}

    def bn_params(name, C):
        if exact:
            out_W[name + ".scale"] = W[name + ".scale"]
            out_W[name + ".shift"] = W[name + ".shift"]
            return W[name + ".scale"], W[name + ".shift"], np.zeros(C, np.float32), np.ones(C, np.float32)
        gamma = (1.0 + 0.2 * rng.standard_normal(C)).astype(np.float32)
        beta = (0.1 * rng.standard_normal(C)).astype(np.float32)
        mean = (0.1 * rng.standard_normal(C)).astype(np.float32)
        var = rng.uniform(0.5, 1.5, C).astype(np.float32)
        s = gamma.astype(np.float64) / np.sqrt(var.astype(np.float64) + np.float64(eps))
        out_W[name + ".scale"] = s.astype(np.float32)
        out_W[name + ".shift"] = (beta.astype(np.float64) - mean.astype(np.float64) * s).astype(np.float32)
        return gamma, beta, mean, var

    def bn_node(x, name, C):
        ga, be, mu, va = bn_params(name, C)
        return g.node("BatchNormalization", [x, g.init(ga), g.init(be), g.init(mu), g.init(va)], epsilon=float(eps))

    def conv_bn(x, wname, bnname, w, **attrs):
        C = w.shape[0]
        if fused and not exact:
            wf = (w * (1.0 + 0.1 * rng.standard_normal((C,) + (1,) * (w.ndim - 1)))).astype(np.float32)
            b = (0.1 * rng.standard_normal(C)).astype(np.float32)
            out_W[wname] = wf
            out_W[bnname + ".scale"] = np.ones(C, np.float32)
            out_W[bnname + ".shift"] = b
            return g.node("Conv", [x, g.init(wf), g.init(b)], **attrs)
        out_W[wname] = w
        y = g.node("Conv", [x, g.init(w)], **attrs)
        return bn_node(y, bnname, C)

    def conv(x, wname, w, bname=None, **attrs):
        out_W[wname] = w
        ins = [x, g.init(w)]
        if bname is not None:
            out_W[bname] = W[bname]
            ins.append(g.init(W[bname]))
        return g.node("Conv", ins, **attrs)

    x = g.node("Unsqueeze", ["feats", g.init(np.array([1]), "i64")])
    x = g.node("Relu", [conv_bn(x, "head.conv1", "head.bn1", W["head.conv1"], pads=[1, 1, 1, 1])])
    for L in (1, 2):
        for b in range(2):
            p = "head.layer%d.%d" % (L, b)
            s = 2 if b == 0 else 1
            y = g.node("Relu", [conv_bn(x, p + ".conv1", p + ".bn1", W[p + ".conv1"], strides=[s, 1])])
            y = conv_bn(y, p + ".conv2", p + ".bn2", W[p + ".conv2"])
            sc = conv_bn(x, p + ".shortcut", p + ".shortcut_bn", W[p + ".shortcut"], strides=[2, 1]) if b == 0 else x
            x = g.node("Relu", [g.node("Add", [y, sc])])
    x = g.node("Relu", [conv_bn(x, "head.conv2", "head.bn2", W["head.conv2"], strides=[2, 1])])
    x = g.node("Reshape", [x, g.init(np.array([0, -1, 0]), "i64")])
    x = g.node("Relu", [conv_bn(x, "tdnn.linear", "tdnn.bn", W["tdnn.linear"], strides=[2], pads=[2, 2])])
    ch = D.INIT_CH
    for bi, (nl, k, dil) in enumerate(D.CAM_BLOCKS):
        for li in range(nl):
            p = "block%d.%d" % (bi + 1, li)
            cin = ch + li * D.GROWTH
            h = g.node("Relu", [bn_node(x, p + ".bn1", cin)])
            h = g.node("Relu", [conv_bn(h, p + ".linear1", p + ".bn2", W[p + ".linear1"])])
            y = conv(h, p + ".local", W[p + ".local"], dilations=[dil], pads=[dil, dil])
            c = g.node("Add", [g.node("ReduceMean", [h], axes=[-1], keepdims=1), g.node("AveragePool", [h])])
            c = g.node("Relu", [conv(c, p + ".cam1.weight", W[p + ".cam1.weight"], p + ".cam1.bias")])
            m = g.node("Sigmoid", [conv(c, p + ".cam2.weight", W[p + ".cam2.weight"], p + ".cam2.bias")])
            x = g.node("Concat", [x, g.node("Mul", [y, m])], axis=1)
        ch += nl * D.GROWTH
        x = g.node("Relu", [bn_node(x, "transit%d.bn" % (bi + 1), ch)])
        x = conv(x, "transit%d.linear" % (bi + 1), W["transit%d.linear" % (bi + 1)])
        ch //= 2
    x = g.node("Relu", [bn_node(x, "out.bn", ch)])
    x = g.node("Concat", [g.node("ReduceMean", [x], axes=[-1], keepdims=0),
                          g.node("ReduceMean", [x], axes=[-1], keepdims=0)], axis=1)   # stats pool (shape only)
    x = g.node("Unsqueeze", [x, g.init(np.array([-1]), "i64")])
    y = conv(x, "dense.linear", W["dense.linear"])
    if fused or exact:   # dense conv + BN(affine=False) fused by the exporter
        if exact:
            assert (W["dense.bn.scale"] == 1).all()
            b = W["dense.bn.shift"]
        else:
            b = (0.1 * rng.standard_normal(512)).astype(np.float32)
        out_W["dense.bn.scale"] = np.ones(512, np.float32)
        out_W["dense.bn.shift"] = b
        g.nodes.pop()   # rebuild the dense conv with the fused bias
        y = g.node("Conv", [x, g.init(out_W["dense.linear"]), g.init(b)])
        y = g.node("Squeeze", [y, g.init(np.array([-1]), "i64")])
    else:
        y = g.node("Squeeze", [y, g.init(np.array([-1]), "i64")])
        y = bn_node(y, "dense.bn", 512)   # affine=False: gamma 1, beta 0 in a real export; seeded here
    with open(path, "wb") as f:
        f.write(g.model("feats", y))
    return out_W


# ---------------------------------------------------------------- Silero VAD (ggml)


def write_silero_ggml(path, seed=3, ftype16=True):
    """whisper.cpp's Silero VAD model file layout (csrc/model_files.cpp load_silero_ggml) with
    the oracle's vad_weights(), mutated; matrices f16 (ftype16) or f32, biases f32."""
    from oracle import vad as V
    W = V.vad_weights()
    rng = np.random.default_rng(seed)
    for k in sorted(W):
        if k == "stft":
            continue
        f = np.float32(rng.uniform(0.8, 1.2))
        W[k] = (W[k].astype(np.float32) * f).astype(W[k].dtype)
    out = bytearray(struct.pack("<I", 0x67676D6C))
    mt = b"silero-16k"
    out += struct.pack("<i", len(mt)) + mt + struct.pack("<3i", 5, 1, 2) + struct.pack("<3i", 512, 64, 4)
    for ci, co in ((129, 128), (128, 64), (64, 64), (64, 128)):
        out += struct.pack("<3i", ci, co, 3)
    out += struct.pack("<4i", 128, 128, 128, 1)
    names = [("_model.stft.forward_basis_buffer", W["stft"].reshape(258, 1, 256))]
    for name, o, i, k, _ in V.CONVS:
        names += [(name + ".weight", W[name + ".weight"]), (name + ".bias", W[name + ".bias"])]
    for n in ("_model.decoder.rnn.weight_ih", "_model.decoder.rnn.weight_hh", "_model.decoder.rnn.bias_ih",
              "_model.decoder.rnn.bias_hh", "_model.decoder.decoder.2.weight", "_model.decoder.decoder.2.bias"):
        names.append((n, W[n]))
    for name, a in names:
        f16 = a.ndim > 1 and ftype16
        data = np.ascontiguousarray(a.astype("<f2" if f16 else "<f4"))
        ne = list(reversed(data.shape))
        nb = name.encode()
        out += struct.pack("<3i", len(ne), len(nb), 1 if f16 else 0) + struct.pack("<%di" % len(ne), *ne) + nb
        out += data.tobytes()
    with open(path, "wb") as f:
        f.write(bytes(out))
    return W
