// hn_cabi_demo: the descriptor forward driven through the C ABI alone (include/hardnet_mi355x.h
// + the HIP runtime; no Python, no torch) -- what a non-Python host binding does.
//
//   hn_cabi_demo <model> <params.f32> <input.f32> <n> <out.f32>
//     model: hardnet | fdl_nasnet | fdl_nasnet01 | nas:o0,o1,o2,o3,o4,o5 (CANDIDATE_BLOCKS indices)
//     params.f32: the module's state_dict floats in order (hardnetnas_amd/_native.py::state_dict_blob)
//     input.f32:  n x 1 x 32 x 32 fp32; out.f32 receives n x 128 fp32
// Exit status 0 on success; on failure the library's hn_last_error() is printed.
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hardnet_mi355x.h"

static bool read_file(const char* path, std::vector<float>& v) {
  FILE* f = std::fopen(path, "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long bytes = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  v.resize((size_t)bytes / sizeof(float));
  const bool ok = std::fread(v.data(), sizeof(float), v.size(), f) == v.size();
  std::fclose(f);
  return ok;
}

static int die(const char* what) {
  std::fprintf(stderr, "hn_cabi_demo: %s: %s\n", what, hn_last_error());
  return 1;
}

int main(int argc, char** argv) {
  if (argc != 6) {
    std::fprintf(stderr, "usage: %s <model> <params.f32> <input.f32> <n> <out.f32>\n", argv[0]);
    return 2;
  }
  // SEARCH_SPACE2 (lookup_table_builder.py:22-45) and the FDLNet IRF layers (des.py)
  static const int ss_in[6] = {32, 32, 32, 64, 64, 128}, ss_out[6] = {32, 32, 64, 64, 128, 128},
                   ss_s[6] = {2, 1, 2, 1, 2, 1};
  static const int fdl_op[3] = {4, 2, 14}, fdl_in[3] = {64, 64, 128}, fdl_out[3] = {64, 128, 128},
                   fdl_s[3] = {1, 2, 1};
  hn_arch_desc d;
  std::memset(&d, 0, sizeof(d));
  d.bn_eps = 1e-5f;
  const char* model = argv[1];
  if (!std::strcmp(model, "hardnet")) {
    d.kind = HN_KIND_HARDNET;
    d.input_norm_eps = 1e-7f;  // hardnet/HardNet.py:308
    d.l2_eps = 1e-10f;         // hardnet/Utils.py:18
  } else if (!std::strcmp(model, "fdl_nasnet") || !std::strcmp(model, "fdl_nasnet01")) {
    d.kind = !std::strcmp(model, "fdl_nasnet") ? HN_KIND_FDL_NASNET : HN_KIND_FDL_NASNET01;
    d.n_layers = 3;
    for (int i = 0; i < 3; ++i) {
      d.op[i] = fdl_op[i];
      d.c_in[i] = fdl_in[i];
      d.c_out[i] = fdl_out[i];
      d.stride[i] = fdl_s[i];
    }
    d.input_norm_eps = 1e-8f;  // FDLNet-master/latency/NASNet/model/des.py:40-47
    d.l2_eps = 0.f;
  } else if (!std::strncmp(model, "nas:", 4)) {
    d.kind = HN_KIND_NAS;
    d.n_layers = 6;
    const char* p = model + 4;
    for (int i = 0; i < 6; ++i) {
      d.op[i] = std::atoi(p);
      d.c_in[i] = ss_in[i];
      d.c_out[i] = ss_out[i];
      d.stride[i] = ss_s[i];
      p = std::strchr(p, ',');
      if (!p && i < 5) {
        std::fprintf(stderr, "hn_cabi_demo: nas needs 6 op indices\n");
        return 2;
      }
      if (p) ++p;
    }
    d.input_norm_eps = -1.f;  // the NAS nets have no input_norm
    d.l2_eps = 0.f;
  } else {
    std::fprintf(stderr, "hn_cabi_demo: unknown model %s\n", model);
    return 2;
  }
  std::vector<float> params, input;
  if (!read_file(argv[2], params) || !read_file(argv[3], input)) {
    std::fprintf(stderr, "hn_cabi_demo: cannot read %s / %s\n", argv[2], argv[3]);
    return 2;
  }
  const long n = std::atol(argv[4]);
  if (n < 0 || input.size() != (size_t)n * 1024) {
    std::fprintf(stderr, "hn_cabi_demo: input holds %zu floats, expected %ld\n", input.size(), n * 1024);
    return 2;
  }
  size_t want = 0;
  if (hn_param_count(&d, &want)) return die("hn_param_count");
  if (want != params.size()) {
    std::fprintf(stderr, "hn_cabi_demo: %zu parameters given, the library expects %zu\n", params.size(), want);
    return 2;
  }
  hn_model* m = nullptr;
  if (hn_create(&d, params.data(), params.size(), &m)) return die("hn_create");
  size_t ws_bytes = 0;
  if (hn_workspace_bytes(m, n, &ws_bytes)) return die("hn_workspace_bytes");
  float *d_in = nullptr, *d_out = nullptr;
  void* d_ws = nullptr;
  hipStream_t st = nullptr;
  if (hipMalloc(&d_in, (n ? n : 1) * 1024 * sizeof(float)) != hipSuccess ||
      hipMalloc(&d_out, (n ? n : 1) * 128 * sizeof(float)) != hipSuccess ||
      hipMalloc(&d_ws, ws_bytes ? ws_bytes : 16) != hipSuccess || hipStreamCreate(&st) != hipSuccess) {
    std::fprintf(stderr, "hn_cabi_demo: device allocation failed\n");
    return 1;
  }
  if (hipMemcpy(d_in, input.data(), input.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
    return 1;
  if (hn_forward(m, d_in, n, d_out, d_ws, ws_bytes, st)) return die("hn_forward");
  std::vector<float> out((size_t)n * 128);
  if (hipStreamSynchronize(st) != hipSuccess ||
      hipMemcpy(out.data(), d_out, out.size() * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess) {
    std::fprintf(stderr, "hn_cabi_demo: HIP error after hn_forward\n");
    return 1;
  }
  FILE* f = std::fopen(argv[5], "wb");
  if (!f || std::fwrite(out.data(), sizeof(float), out.size(), f) != out.size()) return 2;
  std::fclose(f);
  hn_destroy(m);
  (void)hipStreamDestroy(st);
  (void)hipFree(d_in);
  (void)hipFree(d_out);
  (void)hipFree(d_ws);
  std::printf("hn_cabi_demo: %s, %ld patches -> %s\n", model, n, argv[5]);
  return 0;
}
