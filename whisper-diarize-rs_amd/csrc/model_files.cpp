#include "model_files.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <functional>
#include <iterator>
#include <set>
#include <stdexcept>

namespace wdr {

namespace {

[[noreturn]] void bad(const std::string& what, const std::string& why) {
  throw std::runtime_error("failed to load " + what + ": " + why);
}

std::vector<uint8_t> read_file(const std::string& path, const std::string& what) {
  std::ifstream f(path, std::ios::binary);
  if (!f) bad(what, "cannot open " + path);
  return std::vector<uint8_t>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

float half_to_float(uint16_t h) {
  const uint32_t s = (uint32_t)(h & 0x8000) << 16;
  uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ff, u;
  if (e == 0) {
    if (m == 0) {
      u = s;
    } else {
      e = 127 - 15 + 1;
      while (!(m & 0x400)) {
        m <<= 1;
        --e;
      }
      m &= 0x3ff;
      u = s | (e << 23) | (m << 13);
    }
  } else if (e == 31) {
    u = s | 0x7f800000 | (m << 13);
  } else {
    u = s | ((e + 127 - 15) << 23) | (m << 13);
  }
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// ------------------------------------------------------------------ protobuf wire format
const char* kOnnx = "ONNX model";

struct Pb {
  const uint8_t* p;
  const uint8_t* e;
  bool done() const { return p >= e; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int sh = 0;; sh += 7) {
      if (p >= e || sh > 63) bad(kOnnx, "malformed varint");
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << sh;
      if (!(b & 0x80)) return v;
    }
  }
  uint32_t fixed32() {
    if (e - p < 4) bad(kOnnx, "truncated fixed32");
    uint32_t v;
    memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  uint64_t fixed64() {
    if (e - p < 8) bad(kOnnx, "truncated fixed64");
    uint64_t v;
    memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  Pb sub() {
    const uint64_t n = varint();
    if (n > (uint64_t)(e - p)) bad(kOnnx, "truncated length-delimited field");
    Pb s{p, p + n};
    p += n;
    return s;
  }
  std::string str() {
    Pb s = sub();
    return std::string((const char*)s.p, (size_t)(s.e - s.p));
  }
  void skip(int wt) {
    switch (wt) {
      case 0: varint(); break;
      case 1: fixed64(); break;
      case 2: sub(); break;
      case 5: fixed32(); break;
      default: bad(kOnnx, "unsupported wire type " + std::to_string(wt));
    }
  }
};

// repeated scalar fields come packed (wire type 2) or one per key
template <typename F>
void repeated(Pb& pb, int wt, int scalar_wt, F one) {
  if (wt == 2) {
    Pb s = pb.sub();
    while (!s.done()) one(s);
  } else if (wt == scalar_wt) {
    one(pb);
  } else {
    pb.skip(wt);
  }
}

// TensorProto (onnx.proto3): dims 1, data_type 2, float_data 4, int32_data 5, int64_data 7,
// name 8, raw_data 9, double_data 10, external_data 13, data_location 14
OnnxTensor parse_tensor(Pb t, std::string* name) {
  OnnxTensor out;
  int dtype = 0;
  std::vector<float> fd;
  std::vector<int64_t> i32, i64;
  std::vector<double> dd;
  const uint8_t* raw = nullptr;
  size_t raw_n = 0;
  bool external = false;
  while (!t.done()) {
    const uint64_t key = t.varint();
    const int fn = (int)(key >> 3), wt = (int)(key & 7);
    switch (fn) {
      case 1: repeated(t, wt, 0, [&](Pb& s) { out.dims.push_back((int64_t)s.varint()); }); break;
      case 2: dtype = (int)t.varint(); break;
      case 4:
        repeated(t, wt, 5, [&](Pb& s) {
          const uint32_t u = s.fixed32();
          float f;
          memcpy(&f, &u, 4);
          fd.push_back(f);
        });
        break;
      case 5: repeated(t, wt, 0, [&](Pb& s) { i32.push_back((int64_t)(int32_t)s.varint()); }); break;
      case 7: repeated(t, wt, 0, [&](Pb& s) { i64.push_back((int64_t)s.varint()); }); break;
      case 8: *name = t.str(); break;
      case 9: {
        Pb s = t.sub();
        raw = s.p;
        raw_n = (size_t)(s.e - s.p);
        break;
      }
      case 10:
        repeated(t, wt, 1, [&](Pb& s) {
          const uint64_t u = s.fixed64();
          double d;
          memcpy(&d, &u, 8);
          dd.push_back(d);
        });
        break;
      case 13: external = true; t.skip(wt); break;
      case 14: external = external || t.varint() == 1; break;
      default: t.skip(wt);
    }
  }
  if (external) bad(kOnnx, "tensor '" + *name + "' keeps its data in an external file (not supported)");
  const int64_t n = out.numel();
  if (n < 0 || n > (int64_t)1 << 31) bad(kOnnx, "tensor '" + *name + "' has a bad shape");
  auto need = [&](size_t bytes) {
    if (raw_n != bytes) bad(kOnnx, "tensor '" + *name + "' raw_data has " + std::to_string(raw_n) + " bytes, expected " +
                                       std::to_string(bytes));
  };
  out.data.resize((size_t)n);
  switch (dtype) {
    case 1:   // FLOAT
      if (raw) {
        need((size_t)n * 4);
        memcpy(out.data.data(), raw, (size_t)n * 4);
      } else {
        if ((int64_t)fd.size() != n) bad(kOnnx, "tensor '" + *name + "' float_data size");
        out.data = fd;
      }
      break;
    case 10:   // FLOAT16
      for (int64_t k = 0; k < n; ++k) {
        uint16_t h;
        if (raw) {
          need((size_t)n * 2);
          memcpy(&h, raw + 2 * k, 2);
        } else {
          if ((int64_t)i32.size() != n) bad(kOnnx, "tensor '" + *name + "' int32_data size");
          h = (uint16_t)i32[k];
        }
        out.data[k] = half_to_float(h);
      }
      break;
    case 11:   // DOUBLE
      for (int64_t k = 0; k < n; ++k) {
        double d;
        if (raw) {
          need((size_t)n * 8);
          memcpy(&d, raw + 8 * k, 8);
        } else {
          if ((int64_t)dd.size() != n) bad(kOnnx, "tensor '" + *name + "' double_data size");
          d = dd[k];
        }
        out.data[k] = (float)d;
      }
      break;
    case 6:   // INT32
    case 7:   // INT64
      for (int64_t k = 0; k < n; ++k) {
        int64_t v;
        if (raw) {
          if (dtype == 6) {
            need((size_t)n * 4);
            int32_t w;
            memcpy(&w, raw + 4 * k, 4);
            v = w;
          } else {
            need((size_t)n * 8);
            memcpy(&v, raw + 8 * k, 8);
          }
        } else {
          const std::vector<int64_t>& src = dtype == 6 ? i32 : i64;
          if ((int64_t)src.size() != n) bad(kOnnx, "tensor '" + *name + "' integer data size");
          v = src[k];
        }
        out.data[k] = (float)v;
      }
      break;
    default:
      out.data.clear();   // other element types: shape only (never a weight here)
  }
  return out;
}

// AttributeProto: name 1, f 2, i 3, s 4, t 5, floats 7, ints 8
void parse_attr(Pb a, OnnxNode& nd, std::map<std::string, OnnxTensor>* consts) {
  std::string name, sval;
  bool has_f = false, has_i = false, has_s = false, has_t = false;
  double f = 0;
  int64_t i = 0;
  OnnxTensor t;
  while (!a.done()) {
    const uint64_t key = a.varint();
    const int fn = (int)(key >> 3), wt = (int)(key & 7);
    if (fn == 1 && wt == 2) {
      name = a.str();
    } else if (fn == 2 && wt == 5) {
      const uint32_t u = a.fixed32();
      float v;
      memcpy(&v, &u, 4);
      f = v;
      has_f = true;
    } else if (fn == 3 && wt == 0) {
      i = (int64_t)a.varint();
      has_i = true;
    } else if (fn == 4 && wt == 2) {
      sval = a.str();
      has_s = true;
    } else if (fn == 5 && wt == 2) {
      std::string tn;
      t = parse_tensor(a.sub(), &tn);
      has_t = true;
    } else {
      a.skip(wt);
    }
  }
  if (has_f) nd.f[name] = f;
  if (has_i) nd.i[name] = i;
  if (has_s) nd.s[name] = sval;
  if (has_t && nd.op == "Constant" && name == "value" && !nd.out.empty()) (*consts)[nd.out[0]] = t;
  if (has_f && nd.op == "Constant" && name == "value_float" && !nd.out.empty()) {
    OnnxTensor c;
    c.data = {(float)f};
    (*consts)[nd.out[0]] = c;
  }
}

}  // namespace

OnnxModel::OnnxModel(const std::string& path) {
  const std::vector<uint8_t> buf = read_file(path, kOnnx);
  Pb model{buf.data(), buf.data() + buf.size()};
  bool have_graph = false;
  while (!model.done()) {
    const uint64_t key = model.varint();
    const int fn = (int)(key >> 3), wt = (int)(key & 7);
    if (fn != 7 || wt != 2) {
      model.skip(wt);
      continue;
    }
    have_graph = true;
    Pb g = model.sub();
    while (!g.done()) {
      const uint64_t gk = g.varint();
      const int gf = (int)(gk >> 3), gw = (int)(gk & 7);
      if (gf == 1 && gw == 2) {   // NodeProto: input 1, output 2, name 3, op_type 4, attribute 5
        Pb n = g.sub();
        OnnxNode nd;
        std::vector<Pb> attrs;
        while (!n.done()) {
          const uint64_t nk = n.varint();
          const int nf = (int)(nk >> 3), nw = (int)(nk & 7);
          if (nw == 2 && nf == 1) nd.in.push_back(n.str());
          else if (nw == 2 && nf == 2) nd.out.push_back(n.str());
          else if (nw == 2 && nf == 3) nd.name = n.str();
          else if (nw == 2 && nf == 4) nd.op = n.str();
          else if (nw == 2 && nf == 5) attrs.push_back(n.sub());
          else n.skip(nw);
        }
        for (Pb& a : attrs) parse_attr(a, nd, &init);
        nodes.push_back(std::move(nd));
      } else if (gf == 5 && gw == 2) {   // initializer
        std::string name;
        OnnxTensor t = parse_tensor(g.sub(), &name);
        init[name] = std::move(t);
      } else {
        g.skip(gw);
      }
    }
  }
  if (!have_graph) bad(kOnnx, "no graph in " + path);
  // Identity of a constant is that constant (exporters insert them for shared weights)
  for (const OnnxNode& nd : nodes)
    if (nd.op == "Identity" && nd.in.size() == 1 && nd.out.size() == 1 && init.count(nd.in[0]))
      init[nd.out[0]] = init[nd.in[0]];
}

const OnnxTensor* OnnxModel::constant(const std::string& name) const {
  auto it = init.find(name);
  return it == init.end() ? nullptr : &it->second;
}

namespace {

std::string dims_str(const std::vector<int64_t>& d) {
  std::string s = "[";
  for (size_t k = 0; k < d.size(); ++k) s += (k ? "," : "") + std::to_string(d[k]);
  return s + "]";
}

struct Graph {
  const OnnxModel& m;
  std::string what;
  const OnnxTensor& need(const std::string& name, const std::vector<int64_t>& dims, const std::string& role) const {
    const OnnxTensor* t = m.constant(name);
    if (!t) bad(what, role + " ('" + name + "') is not a constant initializer");
    if (t->dims != dims) bad(what, role + " has shape " + dims_str(t->dims) + ", expected " + dims_str(dims));
    return *t;
  }
  // the node producing `v`, following shape-only nodes back to their data input
  const OnnxNode* producer(std::string v) const {
    static const std::set<std::string> shape_only = {"Squeeze", "Unsqueeze", "Reshape", "Flatten", "Identity"};
    for (int hop = 0; hop < 8; ++hop) {
      const OnnxNode* p = nullptr;
      for (const OnnxNode& nd : m.nodes)
        for (const std::string& o : nd.out)
          if (o == v) p = &nd;
      if (!p || !shape_only.count(p->op) || p->in.empty()) return p;
      v = p->in[0];
    }
    return nullptr;
  }
};

// inference BatchNormalization -> per-channel affine (scale, shift), in double as the oracle
// folds it: s = gamma / sqrt(var + eps), t = beta - mean * s
void fold_bn(const Graph& g, const OnnxNode& bn, int64_t C, std::vector<float>* s, std::vector<float>* t) {
  const OnnxTensor& ga = g.need(bn.in.at(1), {C}, "BatchNormalization scale");
  const OnnxTensor& be = g.need(bn.in.at(2), {C}, "BatchNormalization bias");
  const OnnxTensor& mu = g.need(bn.in.at(3), {C}, "BatchNormalization mean");
  const OnnxTensor& va = g.need(bn.in.at(4), {C}, "BatchNormalization var");
  const double eps = bn.f.count("epsilon") ? bn.f.at("epsilon") : 1e-5;
  s->resize(C);
  t->resize(C);
  for (int64_t c = 0; c < C; ++c) {
    const double sc = (double)ga.data[c] / std::sqrt((double)va.data[c] + eps);
    (*s)[c] = (float)sc;
    (*t)[c] = (float)((double)be.data[c] - (double)mu.data[c] * sc);
  }
}

}  // namespace

// ------------------------------------------------------------------ Silero VAD (ggml)
// whisper.cpp's VAD model file, as its converter (models/convert-silero-vad-to-ggml.py) writes
// it and whisper_vad_init_with_params reads it: magic 0x67676d6c, model type (int32 length +
// bytes), version major / minor / patch, window size, context size, encoder layer count, then
// per encoder layer (in, out, kernel), LSTM input and hidden size, final conv in / out (int32
// each), then tensors until EOF in whisper.cpp's record layout (int32 n_dims, name length,
// type 0 f32 / 1 f16, ne[n_dims] innermost first, name, data).  Restated from the published
// converter (whisper.cpp is not in this container): parity of the header layout is unpinned.
TensorMap load_silero_ggml(const std::string& path) {
  const std::string what = "Silero VAD model";
  const std::vector<uint8_t> buf = read_file(path, what);
  const uint8_t* p = buf.data();
  const uint8_t* e = p + buf.size();
  auto i32 = [&]() {
    if (e - p < 4) bad(what, "truncated file");
    int32_t v;
    memcpy(&v, p, 4);
    p += 4;
    return v;
  };
  if ((uint32_t)i32() != 0x67676d6cu) bad(what, "bad magic (not a ggml file): " + path);
  const int32_t tl = i32();
  if (tl < 0 || tl > 256 || e - p < tl) bad(what, "bad model type");
  const std::string type((const char*)p, (size_t)tl);
  p += tl;
  if (type.rfind("silero", 0) != 0) bad(what, "model type '" + type + "' is not a Silero VAD");
  i32(); i32(); i32();   // version
  const int32_t window = i32(), context = i32(), n_enc = i32();
  if (window != 512 || context != 64) bad(what, "window / context " + std::to_string(window) + " / " +
                                                     std::to_string(context) + ", expected 512 / 64 (16 kHz model)");
  const int32_t want_in[4] = {129, 128, 64, 64}, want_out[4] = {128, 64, 64, 128};
  if (n_enc != 4) bad(what, std::to_string(n_enc) + " encoder layers, expected 4");
  for (int l = 0; l < 4; ++l) {
    const int32_t ci = i32(), co = i32(), k = i32();
    if (ci != want_in[l] || co != want_out[l] || k != 3) bad(what, "encoder layer " + std::to_string(l) + " dims");
  }
  const int32_t lin = i32(), lh = i32(), fin = i32(), fout = i32();
  if (lin != 128 || lh != 128 || fin != 128 || fout != 1) bad(what, "LSTM / final conv dims");
  std::map<std::string, std::pair<std::vector<int64_t>, std::vector<float>>> tensors;
  while (p < e) {
    const int32_t nd = i32(), nl = i32(), ty = i32();
    if (nd < 1 || nd > 4 || nl <= 0 || nl > 256 || (ty != 0 && ty != 1)) bad(what, "bad tensor header");
    std::vector<int64_t> ne;
    int64_t n = 1;
    for (int k = 0; k < nd; ++k) {
      // untrusted dimensions: each in [1, 2^24] and the running product bounded by the file
      // size before it is used (no sign games, no overflow)
      const int32_t dk = i32();
      if (dk < 1 || dk > (1 << 24)) bad(what, "bad tensor dimension " + std::to_string(dk));
      ne.push_back(dk);
      n *= dk;
      if (n > (int64_t)buf.size()) bad(what, "tensor larger than the file");
    }
    if (e - p < nl) bad(what, "truncated file");
    const std::string name((const char*)p, (size_t)nl);
    p += nl;
    const size_t bytes = (size_t)n * (ty == 0 ? 4 : 2);
    if ((size_t)(e - p) < bytes) bad(what, "truncated tensor '" + name + "'");
    std::vector<float> v((size_t)n);
    for (int64_t k = 0; k < n; ++k) {
      if (ty == 0) {
        memcpy(&v[k], p + 4 * k, 4);
      } else {
        uint16_t h;
        memcpy(&h, p + 2 * k, 2);
        v[k] = half_to_float(h);
      }
    }
    p += bytes;
    tensors[name] = {ne, std::move(v)};
  }
  TensorMap out;
  auto take = [&](const std::string& file_name, const std::string& key, int64_t n) {
    auto it = tensors.find(file_name);
    if (it == tensors.end()) bad(what, "tensor '" + file_name + "' not found");
    if ((int64_t)it->second.second.size() != n)
      bad(what, "tensor '" + file_name + "' has " + std::to_string(it->second.second.size()) + " elements, expected " +
                    std::to_string(n));
    out[key] = it->second.second;
  };
  take("_model.stft.forward_basis_buffer", "stft", 258 * 256);
  const int co[4] = {128, 64, 64, 128}, ci[4] = {129, 128, 64, 64};
  for (int l = 0; l < 4; ++l) {
    const std::string nm = "_model.encoder." + std::to_string(l) + ".reparam_conv";
    take(nm + ".weight", nm + ".weight", (int64_t)co[l] * ci[l] * 3);
    take(nm + ".bias", nm + ".bias", co[l]);
  }
  for (const char* nm : {"_model.decoder.rnn.weight_ih", "_model.decoder.rnn.weight_hh"}) take(nm, nm, 512 * 128);
  for (const char* nm : {"_model.decoder.rnn.bias_ih", "_model.decoder.rnn.bias_hh"}) take(nm, nm, 512);
  take("_model.decoder.decoder.2.weight", "_model.decoder.decoder.2.weight", 128);
  take("_model.decoder.decoder.2.bias", "_model.decoder.decoder.2.bias", 1);
  return out;
}

// ------------------------------------------------------------------ segmentation-3.0 (ONNX)
// pyannote PyanNet as exported to ONNX (pyannote-rs's segmentation-3.0.onnx): in graph order,
// 4 InstanceNormalization (wav_norm1d, then SincNet's norm1d[0..2]), 3 Conv (the SincNet
// filterbank -- a constant once the exporter folded its parametric filters -- and two k5
// convs), 4 bidirectional LSTM (hidden 128; ONNX gates i, o, f, c reordered to torch's
// i, f, g, o; B = [Wb | Rb]), then 3 linear layers as Gemm or MatMul + Add (linear[0],
// linear[1], classifier).
TensorMap load_segmentation_onnx(const std::string& path) {
  const OnnxModel m(path);
  const Graph g{m, "segmentation model"};
  std::vector<const OnnxNode*> norms, convs, lstms, lins;
  for (const OnnxNode& nd : m.nodes) {
    if (nd.op == "InstanceNormalization") norms.push_back(&nd);
    else if (nd.op == "Conv") convs.push_back(&nd);
    else if (nd.op == "LSTM") lstms.push_back(&nd);
    else if (nd.op == "Gemm" || (nd.op == "MatMul" && nd.in.size() == 2 && m.constant(nd.in[1]))) lins.push_back(&nd);
  }
  if (norms.size() != 4 || convs.size() != 3 || lstms.size() != 4 || lins.size() != 3)
    bad(g.what, "graph has " + std::to_string(norms.size()) + " InstanceNormalization, " + std::to_string(convs.size()) +
                    " Conv, " + std::to_string(lstms.size()) + " LSTM, " + std::to_string(lins.size()) +
                    " linear nodes; segmentation-3.0 has 4 / 3 / 4 / 3");
  TensorMap out;
  const char* nn[4] = {"wav_norm", "norm0", "norm1", "norm2"};
  const int64_t nc[4] = {1, 80, 60, 60};
  for (int k = 0; k < 4; ++k) {
    const OnnxNode& nd = *norms[k];
    const double eps = nd.f.count("epsilon") ? nd.f.at("epsilon") : 1e-5;
    if (std::fabs(eps - 1e-5) > 1e-9) bad(g.what, "InstanceNormalization epsilon " + std::to_string(eps) + " (1e-5 expected)");
    out[std::string(nn[k]) + ".weight"] = g.need(nd.in.at(1), {nc[k]}, "InstanceNormalization scale").data;
    out[std::string(nn[k]) + ".bias"] = g.need(nd.in.at(2), {nc[k]}, "InstanceNormalization bias").data;
  }
  const char* cn[3] = {"sinc", "conv1", "conv2"};
  const std::vector<int64_t> cd[3] = {{80, 1, 251}, {60, 80, 5}, {60, 60, 5}};
  for (int k = 0; k < 3; ++k) {
    const OnnxNode& nd = *convs[k];
    out[std::string(cn[k]) + ".weight"] = g.need(nd.in.at(1), cd[k], "Conv weight").data;
    std::vector<float> b((size_t)cd[k][0], 0.f);
    if (nd.in.size() > 2 && !nd.in[2].empty()) b = g.need(nd.in[2], {cd[k][0]}, "Conv bias").data;
    if (k == 0) {
      for (float v : b)
        if (v != 0.f) bad(g.what, "the SincNet filterbank conv has a nonzero bias");
    } else {
      out[std::string(cn[k]) + ".bias"] = b;
    }
  }
  const int onnx_to_torch[4] = {0, 2, 3, 1};   // torch gate block j <- ONNX block onnx_to_torch[j]
  for (int l = 0; l < 4; ++l) {
    const OnnxNode& nd = *lstms[l];
    const int64_t I = l == 0 ? 60 : 256;
    if (nd.s.count("direction") && nd.s.at("direction") != "bidirectional") bad(g.what, "LSTM is not bidirectional");
    if (nd.i.count("hidden_size") && nd.i.at("hidden_size") != 128) bad(g.what, "LSTM hidden size is not 128");
    const OnnxTensor& W = g.need(nd.in.at(1), {2, 512, I}, "LSTM W");
    const OnnxTensor& R = g.need(nd.in.at(2), {2, 512, 128}, "LSTM R");
    std::vector<float> B(2 * 1024, 0.f);
    if (nd.in.size() > 3 && !nd.in[3].empty()) B = g.need(nd.in[3], {2, 1024}, "LSTM B").data;
    for (int dir = 0; dir < 2; ++dir) {
      const std::string sfx = "_l" + std::to_string(l) + (dir ? "_reverse" : "");
      std::vector<float> wih(512 * I), whh(512 * 128), bih(512), bhh(512);
      for (int j = 0; j < 4; ++j) {
        const int o = onnx_to_torch[j];
        for (int r = 0; r < 128; ++r) {
          const size_t dst = (size_t)j * 128 + r, src = (size_t)o * 128 + r;
          std::copy_n(&W.data[((size_t)dir * 512 + src) * I], I, &wih[dst * I]);
          std::copy_n(&R.data[((size_t)dir * 512 + src) * 128], 128, &whh[dst * 128]);
          bih[dst] = B[(size_t)dir * 1024 + src];
          bhh[dst] = B[(size_t)dir * 1024 + 512 + src];
        }
      }
      out["lstm.weight_ih" + sfx] = wih;
      out["lstm.weight_hh" + sfx] = whh;
      out["lstm.bias_ih" + sfx] = bih;
      out["lstm.bias_hh" + sfx] = bhh;
    }
  }
  const char* ln[3] = {"linear0", "linear1", "classifier"};
  const int64_t lin_in[3] = {256, 128, 128}, lin_out[3] = {128, 128, 7};
  for (int k = 0; k < 3; ++k) {
    const OnnxNode& nd = *lins[k];
    const int64_t I = lin_in[k], O = lin_out[k];
    std::vector<float> w((size_t)(O * I)), b((size_t)O, 0.f);
    if (nd.op == "Gemm") {
      const bool tb = nd.i.count("transB") && nd.i.at("transB") != 0;
      if ((nd.f.count("alpha") && nd.f.at("alpha") != 1.0) || (nd.f.count("beta") && nd.f.at("beta") != 1.0))
        bad(g.what, "Gemm with alpha / beta != 1");
      const OnnxTensor& B = g.need(nd.in.at(1), tb ? std::vector<int64_t>{O, I} : std::vector<int64_t>{I, O}, "Gemm B");
      for (int64_t o = 0; o < O; ++o)
        for (int64_t i = 0; i < I; ++i) w[o * I + i] = tb ? B.data[o * I + i] : B.data[i * O + o];
      if (nd.in.size() > 2 && !nd.in[2].empty()) b = g.need(nd.in[2], {O}, "Gemm C").data;
    } else {   // MatMul(x, W[in][out]) then Add(bias)
      const OnnxTensor& B = g.need(nd.in.at(1), {I, O}, "MatMul weight");
      for (int64_t o = 0; o < O; ++o)
        for (int64_t i = 0; i < I; ++i) w[o * I + i] = B.data[i * O + o];
      bool found = false;
      for (const OnnxNode& a : m.nodes) {
        if (a.op != "Add" || a.in.size() != 2) continue;
        for (int side = 0; side < 2; ++side)
          if (a.in[side] == nd.out.at(0) && m.constant(a.in[1 - side])) {
            b = g.need(a.in[1 - side], {O}, "linear bias").data;
            found = true;
          }
        if (found) break;
      }
      if (!found) bad(g.what, "no bias Add after linear layer " + std::to_string(k));
    }
    out[std::string(ln[k]) + ".weight"] = w;
    out[std::string(ln[k]) + ".bias"] = b;
  }
  return out;
}

// ------------------------------------------------------------------ CAM++ (ONNX)
// wespeaker CAMPPlus as exported to ONNX: its Conv and BatchNormalization nodes in graph
// (= execution) order are matched against the model's parametric layers -- FCM head (conv1/bn1,
// two BasicResBlocks per layer incl. the 1x1 shortcut conv/bn of the first, conv2/bn2), TDNN
// conv/bn, per CAM dense layer bn1 / linear1+bn2 / local / cam linear1 (+bias) / cam linear2
// (+bias), per transit bn / linear, out bn, dense conv/bn.  A conv followed by the BN that reads
// its output is folded (scale, shift + scale * bias); a conv the exporter already fused with its
// BN carries a bias and becomes (1, bias).
TensorMap load_campplus_onnx(const std::string& path) {
  const OnnxModel m(path);
  const Graph g{m, "embedding model"};
  std::vector<const OnnxNode*> ops;
  for (const OnnxNode& nd : m.nodes)
    if (nd.op == "Conv" || nd.op == "BatchNormalization") ops.push_back(&nd);
  size_t at = 0;
  TensorMap out;
  auto next = [&](const char* op, const std::string& layer) -> const OnnxNode& {
    if (at >= ops.size() || ops[at]->op != op)
      bad(g.what, "expected a " + std::string(op) + " node for " + layer + " (parametric node " + std::to_string(at) +
                      " of " + std::to_string(ops.size()) + " is " + (at < ops.size() ? ops[at]->op : "missing") + ")");
    return *ops[at++];
  };
  auto conv_bias = [&](const OnnxNode& c, int64_t O) {
    std::vector<float> b;
    if (c.in.size() > 2 && !c.in[2].empty()) b = g.need(c.in[2], {O}, "Conv bias").data;
    return b;
  };
  // conv + its BN (separate or fused) -> weight, name_bn.scale / .shift
  auto conv_bn = [&](const std::string& name, const std::vector<int64_t>& wd, const std::string& bn_name) {
    const OnnxNode& c = next("Conv", name);
    const int64_t O = wd[0];
    out[name] = g.need(c.in.at(1), wd, "Conv weight of " + name).data;
    const std::vector<float> b = conv_bias(c, O);
    std::vector<float> s, t;
    const OnnxNode* bn = at < ops.size() && ops[at]->op == "BatchNormalization" ? ops[at] : nullptr;
    if (bn && g.producer(bn->in.at(0)) == &c) {
      ++at;
      fold_bn(g, *bn, O, &s, &t);
      for (int64_t o = 0; o < O && !b.empty(); ++o) t[o] = (float)((double)t[o] + (double)s[o] * (double)b[o]);
    } else {
      if (b.empty()) bad(g.what, name + ": no BatchNormalization and no fused bias");
      s.assign((size_t)O, 1.f);
      t = b;
    }
    out[bn_name + ".scale"] = s;
    out[bn_name + ".shift"] = t;
  };
  auto bn_only = [&](const std::string& name, int64_t C) {
    std::vector<float> s, t;
    fold_bn(g, next("BatchNormalization", name), C, &s, &t);
    out[name + ".scale"] = s;
    out[name + ".shift"] = t;
  };
  auto conv_plain = [&](const std::string& name, const std::vector<int64_t>& wd, const std::string& bias_name) {
    const OnnxNode& c = next("Conv", name);
    out[name] = g.need(c.in.at(1), wd, "Conv weight of " + name).data;
    std::vector<float> b = conv_bias(c, wd[0]);
    if (bias_name.empty()) {
      for (float v : b)
        if (v != 0.f) bad(g.what, name + " has a bias (the model's conv has none)");
    } else {
      if (b.empty()) bad(g.what, name + " has no bias");
      out[bias_name] = b;
    }
  };
  const int64_t M = 32;
  conv_bn("head.conv1", {M, 1, 3, 3}, "head.bn1");
  for (int L = 1; L <= 2; ++L)
    for (int b = 0; b < 2; ++b) {
      const std::string p = "head.layer" + std::to_string(L) + "." + std::to_string(b);
      conv_bn(p + ".conv1", {M, M, 3, 3}, p + ".bn1");
      conv_bn(p + ".conv2", {M, M, 3, 3}, p + ".bn2");
      if (b == 0) conv_bn(p + ".shortcut", {M, M, 1, 1}, p + ".shortcut_bn");
    }
  conv_bn("head.conv2", {M, M, 3, 3}, "head.bn2");
  conv_bn("tdnn.linear", {128, 320, 5}, "tdnn.bn");
  const int blocks[3][2] = {{12, 3}, {24, 3}, {16, 3}};
  int64_t ch = 128;
  for (int bi = 0; bi < 3; ++bi) {
    for (int li = 0; li < blocks[bi][0]; ++li) {
      const std::string p = "block" + std::to_string(bi + 1) + "." + std::to_string(li);
      const int64_t cin = ch + li * 32;
      bn_only(p + ".bn1", cin);
      conv_bn(p + ".linear1", {128, cin, 1}, p + ".bn2");
      conv_plain(p + ".local", {32, 128, blocks[bi][1]}, "");
      conv_plain(p + ".cam1.weight", {64, 128, 1}, p + ".cam1.bias");
      conv_plain(p + ".cam2.weight", {32, 64, 1}, p + ".cam2.bias");
    }
    ch += blocks[bi][0] * 32;
    bn_only("transit" + std::to_string(bi + 1) + ".bn", ch);
    conv_plain("transit" + std::to_string(bi + 1) + ".linear", {ch / 2, ch, 1}, "");
    ch /= 2;
  }
  bn_only("out.bn", ch);
  conv_bn("dense.linear", {512, 2 * ch, 1}, "dense.bn");
  if (at != ops.size()) bad(g.what, std::to_string(ops.size() - at) + " Conv / BatchNormalization nodes left unmatched");
  return out;
}

}  // namespace wdr
