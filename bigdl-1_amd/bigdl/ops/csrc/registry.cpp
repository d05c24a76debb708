// Names of the native ops compiled into libbigdl_kernels.so (reported by bigdl.ops.native_status()).
#include <hip/hip_runtime.h>

static const char* kOps[] = {
    "cast", "threshold_fwd_bf16", "threshold_bwd_bf16", "sgd", "adam", "bn_fwd_train", "bn_fwd_infer", "bn_bwd",
    "cross_entropy", "logsoftmax", "conv_fwd_igemm", "conv_dgrad_igemm", "conv_wgrad_igemm",
    "lstm_fwd", "lstm_bwd", "conv_fwd_stats", "bn_fwd_train_partials", "quant_rows", "gemm_i8", "image_crop_flip_norm", "maxpool_fwd", "maxpool_bwd", "bn_fold_partials", "lrn_fwd", "lrn_bwd", "conv_fwd_ldy", "dropout", "w_dgrad_xform",
    "conv_fwd_c4", "pad_channels", "gemm", "transpose_bf16", "colsum_bf16", "rnn_step", "embedding_fwd", "embedding_bwd", "avgpool_fwd",
    "avgpool_bwd", "softmax", "class_nll", "spmm_csr", "trunc_bf16", "nchw_to_nhwc_bf16", "nms", "roi_align", "vml_unary", "vml_binary", "reduce", "depthwise", "layernorm", "adam_dev", "attention", "stream_probe", "resize_bilinear", "pool3d", "split_bf16x3", "conv_fwd_f32out", "bn32",
};

extern "C" __attribute__((visibility("default"))) int bigdl_num_ops() {
  return (int)(sizeof(kOps) / sizeof(kOps[0]));
}

extern "C" __attribute__((visibility("default"))) const char* bigdl_op_name(int i) {
  int n = bigdl_num_ops();
  return (i >= 0 && i < n) ? kOps[i] : "";
}

int g_bigdl_deterministic = 0;

extern "C" __attribute__((visibility("default"))) int bigdl_set_deterministic(int on) {
  g_bigdl_deterministic = on ? 1 : 0;
  return 0;
}

extern "C" __attribute__((visibility("default"))) int bigdl_device_sync() { return (int)hipDeviceSynchronize(); }

// A HIP stream restricted to a subset of the device's compute units (hipExtStreamCreateWithCUMask):
// keep CU i when (i % period) < keep.  Used for the side stream of the asynchronous weight gradients
// so they cannot occupy every CU while the backward-data chain on the step stream waits for slots.
// Returns the stream handle as an integer (0 on failure); wrapped by torch.cuda.ExternalStream.
extern "C" __attribute__((visibility("default"))) long long bigdl_stream_create_cumask(int keep, int period) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return 0;
  const int ncu = prop.multiProcessorCount;
  if (period <= 0 || keep <= 0 || keep > period || ncu <= 0 || ncu > 1024) return 0;
  uint32_t mask[32] = {0};
  for (int i = 0; i < ncu; ++i)
    if (i % period < keep) mask[i / 32] |= 1u << (i % 32);
  hipStream_t s = nullptr;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)((ncu + 31) / 32), mask) != hipSuccess) return 0;
  return (long long)(intptr_t)s;
}
