// Python bindings of the native extension ``_C`` (kernels launch on torch's current HIP
// stream so they compose with RCCL collectives and hipGraph capture).
#include <torch/extension.h>
#include <pybind11/stl.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>

#include <memory>
#include <string>
#include <vector>

#include "kernels/api.h"
#include "kernels/stamps.h"
#include "runtime/mailbox.h"

namespace py = pybind11;

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_f32_cuda(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void adam_flat(at::Tensor w, at::Tensor g, at::Tensor m, at::Tensor v, double lr_t, double b1,
               double b2, double eps, double scale) {
  check_f32_cuda(w, "w");
  check_f32_cuda(g, "g");
  check_f32_cuda(m, "m");
  check_f32_cuda(v, "v");
  const int64_t n = w.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n && v.numel() == n, "adam_flat: size mismatch");
  ddl::launch_adam(w.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(),
                   v.data_ptr<float>(), n, (float)lr_t, (float)b1, (float)b2, (float)eps,
                   (float)scale, cur_stream());
}

void momentum_flat(at::Tensor w, at::Tensor g, at::Tensor m, double lr, double mu, double scale) {
  check_f32_cuda(w, "w");
  check_f32_cuda(g, "g");
  check_f32_cuda(m, "m");
  const int64_t n = w.numel();
  TORCH_CHECK(g.numel() == n && m.numel() == n, "momentum_flat: size mismatch");
  ddl::launch_momentum(w.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), n,
                       (float)lr, (float)mu, (float)scale, cur_stream());
}

// Python-facing wrapper of ddl::Engine: owns the workspace tensor.
class PyEngine {
 public:
  PyEngine(std::vector<at::Tensor> params, std::vector<at::Tensor> grads, int64_t max_batch,
           int64_t train_batch, double keep_prob)
      : params_(params), grads_(grads) {
    TORCH_CHECK(params.size() == 14 && grads.size() == 14, "need 14 parameter/gradient tensors");
    for (int i = 0; i < 14; ++i) {
      check_f32_cuda(params[i], "param");
      check_f32_cuda(grads[i], "grad");
      e_.P[i] = params[i].data_ptr<float>();
      e_.G[i] = grads[i].data_ptr<float>();
    }
    device_ = params[0].device();
    e_.max_batch = (int)std::max(max_batch, train_batch);
    e_.train_batch = (int)train_batch;
    set_keep_prob(keep_prob);
    realloc();
  }

  void set_cfg(std::vector<int64_t> c) {
    TORCH_CHECK((int)c.size() == ddl::OP_COUNT, "expected ", (int)ddl::OP_COUNT, " tile configs");
    for (int i = 0; i < ddl::OP_COUNT; ++i) {
      TORCH_CHECK((c[i] >= 0 && c[i] < ddl::NUM_TILE_CFGS) || c[i] == ddl::CFG_KWAVE ||
                      c[i] == ddl::CFG_MF16 || c[i] == ddl::CFG_KW16,
                  "tile config out of range");
      e_.cfg[i] = (int)c[i];
    }
    realloc();
  }
  std::vector<int64_t> get_cfg() const {
    return std::vector<int64_t>(e_.cfg, e_.cfg + ddl::OP_COUNT);
  }
  // tile configs of the eval forward (no split-K, large batch chunks); no slab needed
  void set_eval_cfg(std::vector<int64_t> c) {
    TORCH_CHECK((int)c.size() == ddl::OP_COUNT, "expected ", (int)ddl::OP_COUNT, " tile configs");
    for (int i = 0; i < ddl::OP_COUNT; ++i) {
      // the eval-only large tiles exist for the conv2-4 forward ops only
      const bool big = i == ddl::OP_CONV2_FWD || i == ddl::OP_CONV3_FWD || i == ddl::OP_CONV4_FWD;
      // (CFG_KWAVE: the K-wave launch; ops without a K-wave instantiation fall back to the
      // one-wave 32x32 tile, engine_impl.h launch_cfg)
      TORCH_CHECK(c[i] == ddl::CFG_KWAVE ||
                      (c[i] >= 0 && c[i] < (big ? ddl::NUM_EVAL_TILE_CFGS : ddl::NUM_TILE_CFGS)),
                  "tile config out of range");
      e_.eval_cfg[i] = (int)c[i];
    }
  }
  std::vector<int64_t> get_eval_cfg() const {
    return std::vector<int64_t>(e_.eval_cfg, e_.eval_cfg + ddl::OP_COUNT);
  }
  // the side stream exists only in the (slower, A/B) two-stream mode: every extra HIP stream
  // competes for the GPU_MAX_HW_QUEUES hardware queues
  void set_concurrent(bool on) {
    if (on) {
      c10::hip::HIPGuard guard(device_.index());
      e_.init_streams();
    }
    e_.concurrent = on;
  }
  void set_dual(bool on) { e_.dual = on; }
  void set_wide_thr(int64_t t) {
    e_.wide_thr = (int)std::max<int64_t>(1, t);
    for (int i = 0; i < ddl::OP_COUNT; ++i) e_.wide[i] = e_.wide_thr;
  }
  // per-op split-K reduce threshold: z > wide[op] -> separate reduce kernel, else in-launch
  void set_wide(std::vector<int64_t> w) {
    TORCH_CHECK((int)w.size() == ddl::OP_COUNT, "expected ", (int)ddl::OP_COUNT, " thresholds");
    for (int i = 0; i < ddl::OP_COUNT; ++i) e_.wide[i] = (int)std::max<int64_t>(1, w[i]);
  }
  std::vector<int64_t> get_wide() const {
    return std::vector<int64_t>(e_.wide, e_.wide + ddl::OP_COUNT);
  }
  // bit op: the dual launch of op's layer dispatches its second problem first
  void set_dual_bfirst(int64_t m) { e_.dual_bfirst = (int)m; }
  int64_t get_dual_bfirst() const { return e_.dual_bfirst; }

  void set_keep_prob(double keep) {
    const double rate = 1.0 - keep;
    e_.thr24 = (uint32_t)std::llround(rate * 16777216.0);
    e_.inv_keep = keep > 0.0 ? (float)(1.0 / keep) : 0.f;
  }

  void set_splits(std::vector<int64_t> s) {
    TORCH_CHECK((int)s.size() == ddl::OP_COUNT, "expected ", (int)ddl::OP_COUNT, " split factors");
    for (int i = 0; i < ddl::OP_COUNT; ++i) e_.splits[i] = (int)std::max<int64_t>(1, s[i]);
    realloc();
  }
  std::vector<int64_t> get_splits() const {
    return std::vector<int64_t>(e_.splits, e_.splits + ddl::OP_COUNT);
  }
  void forward(at::Tensor x, at::Tensor seed, bool train) {
    check_x(x);
    e_.forward(x.data_ptr<float>(), (int)x.size(0), seed_ptr(seed), train, cur_stream());
  }
  void backward_segment(int64_t s, at::Tensor x, at::Tensor labels, at::Tensor seed) {
    check_x(x);
    TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_cuda(), "labels must be int64 GPU");
    e_.backward_segment((int)s, x.data_ptr<float>(), labels.data_ptr<int64_t>(), (int)x.size(0),
                        seed_ptr(seed), cur_stream());
  }
  void run_op(int64_t op, at::Tensor x, at::Tensor seed, bool train) {
    check_x(x);
    e_.run_op((int)op, x.data_ptr<float>(), (int)x.size(0), seed_ptr(seed), train, cur_stream());
  }
  void zero_correct() {
    TORCH_CHECK(hipMemsetAsync(e_.correct, 0, sizeof(int), cur_stream()) == hipSuccess);
  }
  void eval_count(at::Tensor x, at::Tensor labels) {
    check_x(x);
    e_.eval_count(x.data_ptr<float>(), labels.data_ptr<int64_t>(), (int)x.size(0), cur_stream());
  }
  void head_fwd(at::Tensor labels, int64_t B) {
    ddl::launch_head_fwd(e_.h2, e_.P[12], e_.P[13], labels.data_ptr<int64_t>(), (int)B, e_.dlog,
                         e_.loss, nullptr, cur_stream());
  }

  // Views of internal buffers (testing / debugging).  Shapes are for batch B.
  at::Tensor buffer(const std::string& name, int64_t B) {
    auto f = at::TensorOptions().dtype(at::kFloat).device(device_);
    auto u8 = at::TensorOptions().dtype(at::kByte).device(device_);
    auto i32 = at::TensorOptions().dtype(at::kInt).device(device_);
    // maps stored with the 2-pixel zero halo (layers.h kHalo): the interior view
    // ("p1+halo" etc.: the whole stored map, border included)
    const bool whole = name.size() > 5 && name.compare(name.size() - 5, 5, "+halo") == 0;
    const std::string base_name = whole ? name.substr(0, name.size() - 5) : name;
    auto halo = [&](float* p, int64_t h, int64_t c) {
      auto t = torch::from_blob(p, {B, h + 4, h + 4, c}, f);
      return whole ? t : t.narrow(1, 2, h).narrow(2, 2, h);
    };
    if (whole && base_name == "p1") return halo(e_.p1, 14, 32);
    if (whole && base_name == "p2") return halo(e_.p2, 7, 64);
    if (whole && base_name == "p3") return halo(e_.p3, 4, 128);
    if (whole && base_name == "d4") return halo(e_.d4, 4, 256);
    if (whole && base_name == "d3") return halo(e_.d3, 7, 128);
    if (whole && base_name == "d2") return halo(e_.d2, 14, 64);
    if (name == "p1") return halo(e_.p1, 14, 32);
    if (name == "p2") return halo(e_.p2, 7, 64);
    if (name == "p3") return halo(e_.p3, 4, 128);
    if (name == "p4") return torch::from_blob(e_.p4, {B, 1024}, f);
    if (name == "h1") return torch::from_blob(e_.h1, {B, 1024}, f);
    if (name == "h2") return torch::from_blob(e_.h2, {B, 512}, f);
    if (name == "dlog") return torch::from_blob(e_.dlog, {B, 10}, f);
    if (name == "loss") return torch::from_blob(e_.loss, {B}, f);
    if (name == "dpre2fc") return torch::from_blob(e_.dpre2fc, {B, 512}, f);
    if (name == "dpre1fc") return torch::from_blob(e_.dpre1fc, {B, 1024}, f);
    if (name == "d4") return halo(e_.d4, 4, 256);
    if (name == "d3") return halo(e_.d3, 7, 128);
    if (name == "d2") return halo(e_.d2, 14, 64);
    if (name == "d1") return torch::from_blob(e_.d1, {B, 28, 28, 32}, f);
    if (name == "c1") return torch::from_blob(e_.c1, {B, 14, 14, 32}, u8);
    if (name == "c2") return torch::from_blob(e_.c2, {B, 7, 7, 64}, u8);
    if (name == "c3") return torch::from_blob(e_.c3, {B, 4, 4, 128}, u8);
    if (name == "c4") return torch::from_blob(e_.c4, {B, 1024}, u8);
    if (name == "correct") return torch::from_blob(e_.correct, {1}, i32);
    TORCH_CHECK(false, "unknown buffer ", name);
  }

  int64_t max_batch() const { return e_.max_batch; }
  ddl::Engine* raw() { return &e_; }
  void check_batch(const at::Tensor& x) { check_x(x); }
  int64_t workspace_bytes() const { return (int64_t)e_.workspace_bytes(); }
  static std::vector<int64_t> op_shape(int64_t op, int64_t B) {
    int M, N, K;
    ddl::Engine::op_shape((int)op, (int)B, &M, &N, &K);
    return {M, N, K};
  }

 private:
  void realloc() {
    e_.slab_floats = e_.slab_floats_needed(e_.train_batch);
    const size_t bytes = e_.workspace_bytes();
    // zeroed once: the split-K arrival tickets must start at 0 (reducers re-arm them)
    ws_ = at::zeros({(int64_t)bytes}, at::TensorOptions().dtype(at::kByte).device(device_));
    e_.bind_workspace(ws_.data_ptr());
  }
  void check_x(const at::Tensor& x) {
    check_f32_cuda(x, "x");
    TORCH_CHECK(x.dim() == 2 && x.size(1) == 784, "x must be [B,784]");
    TORCH_CHECK(x.size(0) <= e_.max_batch, "batch ", x.size(0), " exceeds engine max_batch ",
                e_.max_batch);
  }
  static const uint32_t* seed_ptr(const at::Tensor& s) {
    if (!s.defined() || s.numel() == 0) return nullptr;
    TORCH_CHECK(s.is_cuda() && s.scalar_type() == at::kInt, "seed must be an int32 GPU tensor");
    return reinterpret_cast<const uint32_t*>(s.data_ptr<int32_t>());
  }

  ddl::Engine e_;
  std::vector<at::Tensor> params_, grads_;
  at::Tensor ws_;
  at::Device device_{at::kCPU};
};

// Python-facing wrapper of ddl::SyncRunner (native sync step: engine + exchange + update).
// xGMI peer exchange (kernels/xgmi.hip): IPC handles out, every rank's handles in.
class PyPeer {
 public:
  PyPeer(at::Tensor params, at::Tensor grads, int64_t world, int64_t rank, py::list buckets,
         int64_t max_slices, int64_t repl_bucket)
      : params_(params), grads_(grads) {
    check_f32_cuda(params, "params");
    check_f32_cuda(grads, "grads");
    TORCH_CHECK(params.numel() == grads.numel(), "params/grads size mismatch");
    // each bucket: (lo, hi) — an equal-chunk bucket — or (runs, state_offs, owner) — an owner
    // bucket of a tensor-granular plan (kernels/api.h XgmiBucketSpec)
    std::vector<ddl::XgmiBucketSpec> bk;
    for (auto b : buckets) {
      auto t = b.cast<py::tuple>();
      ddl::XgmiBucketSpec sp;
      if (t.size() == 3) {
        for (auto r : t[0].cast<py::list>()) {
          auto rr = r.cast<py::tuple>();
          sp.runs.emplace_back(rr[0].cast<int64_t>(), rr[1].cast<int64_t>());
        }
        sp.state_offs = t[1].cast<std::vector<int64_t>>();
        sp.owner = t[2].cast<int>();
      } else {
        sp.runs.emplace_back(t[0].cast<int64_t>(), t[1].cast<int64_t>());
      }
      bk.push_back(sp);
    }
    c10::hip::HIPGuard guard(params.device().index());
    p_ = std::make_unique<ddl::PeerExchange>(params.data_ptr<float>(), grads.data_ptr<float>(),
                                             params.numel(), (int)world, (int)rank, bk,
                                             (int)max_slices, (int)repl_bucket);
  }
  py::bytes handle() const {
    c10::hip::HIPGuard guard(params_.device().index());
    return py::bytes(p_->handle());
  }
  void open(std::vector<std::string> handles) {
    c10::hip::HIPGuard guard(params_.device().index());
    p_->open(handles);
  }
  int error() const { return p_->error(); }
  std::vector<int64_t> nslices() const {
    std::vector<int64_t> v;
    for (int b = 0; b < p_->num_buckets(); ++b) v.push_back(p_->nslices(b));
    return v;
  }
  void close() {
    c10::hip::HIPGuard guard(params_.device().index());
    py::gil_scoped_release nogil;
    p_->close();
  }
  // -1: equal-chunk bucket; else the rank hosting the owner bucket's PS
  int owner(int64_t b) const {
    TORCH_CHECK(b >= 0 && b < p_->num_buckets(), "bucket out of range");
    return p_->owner((int)b);
  }
  ddl::PeerExchange* raw() { return p_.get(); }

 private:
  at::Tensor params_, grads_;
  std::unique_ptr<ddl::PeerExchange> p_;
};

// asynchronous PS over xGMI peer memory (kernels/xgmi_async.hip); kernels on the current stream
class PyAsyncPeer {
 public:
  PyAsyncPeer(at::Tensor params, at::Tensor grads, int64_t world, int64_t rank, py::list ranges,
              std::vector<int64_t> hosts, int64_t max_slices)
      : params_(params), grads_(grads) {
    check_f32_cuda(params, "params");
    check_f32_cuda(grads, "grads");
    TORCH_CHECK(params.numel() == grads.numel(), "params/grads size mismatch");
    std::vector<std::pair<int64_t, int64_t>> rg;
    for (auto r : ranges) {
      auto t = r.cast<py::tuple>();
      rg.emplace_back(t[0].cast<int64_t>(), t[1].cast<int64_t>());
    }
    std::vector<int> h(hosts.begin(), hosts.end());
    c10::hip::HIPGuard guard(params.device().index());
    p_ = std::make_unique<ddl::AsyncPeer>(params.data_ptr<float>(), grads.data_ptr<float>(),
                                          params.numel(), (int)world, (int)rank, rg, h,
                                          (int)max_slices);
  }
  py::bytes handle() const {
    c10::hip::HIPGuard guard(params_.device().index());
    return py::bytes(p_->handle());
  }
  void open(std::vector<std::string> handles) {
    c10::hip::HIPGuard guard(params_.device().index());
    p_->open(handles);
  }
  void push_all(int64_t epoch, double coef) { p_->push_all((uint32_t)epoch, (float)coef, cur_stream()); }
  void attach_done(std::string name, bool create) { p_->attach_done(name, create); }
  bool wait_done(int64_t epoch, double timeout_s) {
    py::gil_scoped_release nogil;
    return p_->wait_done((uint32_t)epoch, timeout_s);
  }
  // opt: 0 Adam (lr_t, b1, b2, eps), 1 momentum (lr, mu), 2 self-test
  void apply(int64_t ps, int64_t worker, int64_t epoch, int64_t opt, at::Tensor ps_params,
             c10::optional<at::Tensor> m, c10::optional<at::Tensor> v, double lr_t, double b1,
             double b2, double eps, double lr, double mu, double scale) {
    check_f32_cuda(ps_params, "ps_params");
    ddl::XgmiUpdate u;
    u.opt = (int)opt;
    if (m) { check_f32_cuda(*m, "m"); u.m = m->data_ptr<float>(); }
    if (v) { check_f32_cuda(*v, "v"); u.v = v->data_ptr<float>(); }
    u.lr_t = (float)lr_t;
    u.c1 = 1.f - (float)b1;
    u.c2 = 1.f - (float)b2;
    u.eps = (float)eps;
    u.lr = (float)lr;
    u.mu = (float)mu;
    u.scale = (float)scale;
    p_->apply((int)ps, (int)worker, (uint32_t)epoch, u, ps_params.data_ptr<float>(), cur_stream());
  }
  void close() {
    c10::hip::HIPGuard guard(params_.device().index());
    py::gil_scoped_release nogil;
    p_->close();
  }
  int error() const { return p_->error(); }
  ddl::AsyncPeer* raw() { return p_.get(); }
  int device() const { return params_.device().index(); }

 private:
  at::Tensor params_, grads_;
  std::unique_ptr<ddl::AsyncPeer> p_;
};

// native PS service thread of the async xGMI exchange
class PyAsyncService {
 public:
  // ps: list of (ps id, params, m, v | None, t)
  PyAsyncService(PyAsyncPeer& peer, int64_t world, py::list ps, int64_t opt,
                 double lr, double b1, double b2, double eps, double mu, double scale,
                 int64_t epoch0, bool provenance) {
    std::vector<ddl::AsyncPsState> st;
    for (auto item : ps) {
      auto t = item.cast<py::tuple>();
      ddl::AsyncPsState s;
      s.ps = t[0].cast<int>();
      at::Tensor w = t[1].cast<at::Tensor>(), m = t[2].cast<at::Tensor>();
      check_f32_cuda(w, "ps params");
      check_f32_cuda(m, "m");
      keep_.push_back(w);
      keep_.push_back(m);
      s.params = w.data_ptr<float>();
      s.m = m.data_ptr<float>();
      s.v = nullptr;
      if (!t[3].is_none()) {
        at::Tensor v = t[3].cast<at::Tensor>();
        check_f32_cuda(v, "v");
        keep_.push_back(v);
        s.v = v.data_ptr<float>();
      }
      s.t = t[4].cast<int64_t>();
      st.push_back(s);
    }
    svc_ = std::make_unique<ddl::AsyncService>(peer.raw(), (int)world, peer.device(), st,
                                               (int)opt, (float)lr, (float)b1, (float)b2,
                                               (float)eps, (float)mu, (float)scale,
                                               (uint32_t)epoch0, provenance);
  }
  void start(int64_t expected) { svc_->start(expected); }
  void join() {
    py::gil_scoped_release nogil;
    svc_->join();
  }
  int64_t t(int64_t ps) const { return svc_->t((int)ps); }
  int64_t served() const { return svc_->served(); }
  void pause() {
    py::gil_scoped_release nogil;
    svc_->pause();
  }
  void resume() { svc_->resume(); }
  std::vector<std::array<int64_t, 4>> provenance() const { return svc_->provenance(); }
  std::string mode() const { return svc_->mode(); }

 private:
  std::vector<at::Tensor> keep_;
  std::unique_ptr<ddl::AsyncService> svc_;
};

// asynchronous PS over point-to-point RCCL sessions (kernels/rccl_async.hip)
class PyRcclAsync {
 public:
  // ps: list of (ps id, private params, m, v | None, t); ranges: [(lo, hi)] per PS
  PyRcclAsync(at::Tensor params, at::Tensor grads, int64_t world, int64_t rank, py::list ranges,
              std::vector<int64_t> hosts, py::list ps, int64_t opt, double lr, double b1,
              double b2, double eps, double mu, bool self_sessions)
      : params_(params), grads_(grads) {
    check_f32_cuda(params, "params");
    check_f32_cuda(grads, "grads");
    std::vector<std::pair<int64_t, int64_t>> rg;
    for (auto r : ranges) {
      auto t = r.cast<py::tuple>();
      rg.emplace_back(t[0].cast<int64_t>(), t[1].cast<int64_t>());
    }
    std::vector<ddl::AsyncPsState> st;
    for (auto item : ps) {
      auto t = item.cast<py::tuple>();
      ddl::AsyncPsState s;
      s.ps = t[0].cast<int>();
      at::Tensor w = t[1].cast<at::Tensor>(), m = t[2].cast<at::Tensor>();
      check_f32_cuda(w, "ps params");
      check_f32_cuda(m, "m");
      keep_.push_back(w);
      keep_.push_back(m);
      s.params = w.data_ptr<float>();
      s.m = m.data_ptr<float>();
      s.v = nullptr;
      if (!t[3].is_none()) {
        at::Tensor v = t[3].cast<at::Tensor>();
        check_f32_cuda(v, "v");
        keep_.push_back(v);
        s.v = v.data_ptr<float>();
      }
      s.t = t[4].cast<int64_t>();
      st.push_back(s);
    }
    std::vector<int> h(hosts.begin(), hosts.end());
    c10::hip::HIPGuard guard(params.device().index());
    r_ = std::make_unique<ddl::RcclAsync>(params.data_ptr<float>(), grads.data_ptr<float>(),
                                          (int)world, (int)rank, params.device().index(), rg, h,
                                          st, (int)opt, lr, b1, b2, (float)eps, (float)mu,
                                          self_sessions);
  }
  void init_comm(py::bytes id) {
    std::string s = id;
    TORCH_CHECK(s.size() == 128, "RCCL unique id must be 128 bytes");
    py::gil_scoped_release nogil;  // collective
    r_->init_comm(s.data());
  }
  void attach_shm(std::string job, bool create) { r_->attach_shm(job, create); }
  void open_boxes(bool own) { r_->open_boxes(own); }
  void start(int64_t expected, bool provenance) { r_->start(expected, provenance); }
  void push_pull() {
    hipStream_t st = cur_stream();
    py::gil_scoped_release nogil;
    r_->push_pull(st);
  }
  void join() {
    py::gil_scoped_release nogil;
    r_->join();
  }
  void pause() {
    py::gil_scoped_release nogil;
    r_->pause();
  }
  void resume() { r_->resume(); }
  int64_t t(int64_t ps) const { return r_->t((int)ps); }
  void set_t(int64_t ps, int64_t t) { r_->set_t((int)ps, t); }
  int64_t served() const { return r_->served(); }
  std::vector<std::array<int64_t, 4>> provenance() const { return r_->provenance(); }

 private:
  at::Tensor params_, grads_;
  std::vector<at::Tensor> keep_;
  std::unique_ptr<ddl::RcclAsync> r_;
};

// native async worker step (kernels/async_runner.hip)
class PyAsyncRunner {
 public:
  PyAsyncRunner(PyEngine& eng, PyAsyncPeer& peer, int64_t world, int64_t rank,
                std::vector<int64_t> seg_of_ps, int64_t epoch0)
      : eng_(eng) {
    std::vector<int> seg(seg_of_ps.begin(), seg_of_ps.end());
    c10::hip::HIPGuard guard(peer.device());
    r_ = std::make_unique<ddl::AsyncRunner>(eng.raw(), peer.raw(), (int)world, (int)rank,
                                            peer.device(), seg, (uint32_t)epoch0);
  }
  void step(at::Tensor x, at::Tensor labels, int64_t seed, double timeout_s) {
    eng_.check_batch(x);
    TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_cuda(), "labels must be int64 GPU");
    TORCH_CHECK(labels.numel() == x.size(0), "labels/batch size mismatch");
    const float* xp = x.data_ptr<float>();
    const int64_t* lp = labels.data_ptr<int64_t>();
    const int B = (int)x.size(0);
    hipStream_t st = cur_stream();
    py::gil_scoped_release nogil;  // the host wait for the previous round
    r_->step(xp, lp, B, (uint32_t)(seed & 0xFFFFFFFF), st, timeout_s);
  }
  void finish(double timeout_s) {
    py::gil_scoped_release nogil;
    r_->finish(timeout_s);
  }
  int64_t epoch() const { return r_->epoch(); }
  void set_use_tail(bool on) { r_->set_use_tail(on); }
  void set_gate(bool on) { r_->set_gate(on); }
  // ps: list of (ps id, private params, m, v, t), every PS (W = 1, Adam)
  void set_inline(py::list ps, double lr, double b1, double b2, double eps, double scale,
                  bool provenance) {
    std::vector<ddl::AsyncPsState> st;
    for (auto item : ps) {
      auto t = item.cast<py::tuple>();
      ddl::AsyncPsState s;
      s.ps = t[0].cast<int>();
      at::Tensor w = t[1].cast<at::Tensor>(), m = t[2].cast<at::Tensor>();
      TORCH_CHECK(!t[3].is_none(), "in-line applies are Adam: v required");
      at::Tensor v = t[3].cast<at::Tensor>();
      check_f32_cuda(w, "ps params");
      check_f32_cuda(m, "m");
      check_f32_cuda(v, "v");
      keep_.push_back(w);
      keep_.push_back(m);
      keep_.push_back(v);
      s.params = w.data_ptr<float>();
      s.m = m.data_ptr<float>();
      s.v = v.data_ptr<float>();
      s.t = t[4].cast<int64_t>();
      st.push_back(s);
    }
    r_->set_inline(st, (float)lr, (float)b1, (float)b2, (float)eps, (float)scale, provenance);
  }
  bool inline_on() const { return r_->inline_on(); }
  int64_t inline_t(int64_t ps) const { return r_->inline_t((int)ps); }
  void inline_sync_ps() { r_->inline_sync_ps(cur_stream()); }
  std::vector<std::array<int64_t, 4>> inline_provenance() const { return r_->inline_provenance(); }

 private:
  PyEngine& eng_;
  std::vector<at::Tensor> keep_;
  std::unique_ptr<ddl::AsyncRunner> r_;
};

class PyRunner {
 public:
  PyRunner(PyEngine& eng, at::Tensor params, at::Tensor grads, int64_t world, int64_t rank)
      : eng_(eng), params_(params), grads_(grads), world_(world) {
    check_f32_cuda(params, "params");
    check_f32_cuda(grads, "grads");
    TORCH_CHECK(params.numel() == grads.numel(), "params/grads size mismatch");
    r_ = std::make_unique<ddl::SyncRunner>(eng.raw(), params.data_ptr<float>(),
                                           grads.data_ptr<float>(), (int)world, (int)rank);
  }
  static py::bytes unique_id() {
    char id[128];
    ddl::SyncRunner::unique_id(id);
    return py::bytes(id, 128);
  }
  static std::string probe() { return ddl::SyncRunner::probe(); }
  void init_comm(py::bytes id, bool force) {
    std::string s = id;
    TORCH_CHECK(s.size() == 128, "RCCL unique id must be 128 bytes");
    py::gil_scoped_release nogil;  // collective: blocks until every rank joins
    r_->init_comm(s.data(), force);
  }
  bool has_comm() const { return r_->has_comm(); }
  void set_peer(PyPeer& p) {
    peer_keep_ = &p;
    r_->set_peer(p.raw());
  }
  // all buckets with w := sum over ranks of g (the xGMI self-test; blocks until done)
  void peer_selftest_step() {
    py::gil_scoped_release nogil;
    r_->peer_selftest_step(cur_stream());
    (void)hipStreamSynchronize(cur_stream());
  }
  // units: list of (seg, kind, host, ps, [(lo, hi, state_off)], m|None, v|None, shard|None
  //                 [, bucket])
  void set_units(py::list units) {
    std::vector<ddl::RunnerUnit> out;
    keep_.clear();
    const int64_t n = params_.numel();
    for (auto item : units) {
      auto t = item.cast<py::tuple>();
      TORCH_CHECK(t.size() == 8 || t.size() == 9, "unit tuple must have 8 or 9 fields");
      ddl::RunnerUnit u;
      u.seg = t[0].cast<int>();
      u.kind = t[1].cast<int>();
      u.host = t[2].cast<int>();
      u.ps = t[3].cast<int>();
      auto opt_ptr = [&](py::handle h, int64_t need, const char* what) -> float* {
        if (h.is_none()) return nullptr;
        at::Tensor x = h.cast<at::Tensor>();
        check_f32_cuda(x, what);
        TORCH_CHECK(x.numel() >= need, what, " too small");
        keep_.push_back(x);
        return x.data_ptr<float>();
      };
      int64_t need_state = 0, need_shard = 0;
      if (t.size() == 9) u.bucket = t[8].cast<int>();
      // an xGMI OWNER bucket (tensor-granular plan): its owner updates the whole unit
      const bool owner_bucket = u.kind == ddl::RunnerUnit::XGMI && r_->peer() &&
                                u.bucket >= 0 && u.bucket < r_->peer()->num_buckets() &&
                                r_->peer()->owner(u.bucket) >= 0;
      for (auto r : t[4].cast<py::list>()) {
        auto rr = r.cast<py::tuple>();
        ddl::RunnerRange range{rr[0].cast<int64_t>(), rr[1].cast<int64_t>(), rr[2].cast<int64_t>()};
        TORCH_CHECK(0 <= range.lo && range.lo <= range.hi && range.hi <= n, "range out of bounds");
        int64_t len = range.hi - range.lo;
        if (u.kind == ddl::RunnerUnit::RS ||
            (u.kind == ddl::RunnerUnit::XGMI && !owner_bucket)) {  // (AR and
          // XGMI_REPL update the whole range on every rank: state for all of it)
          // reduce-scatter: this rank updates (and needs state / a shard buffer for) 1/W of it;
          // a remainder would silently get no exchange and no update
          TORCH_CHECK(len % world_ == 0, "RS unit range [", range.lo, ", ", range.hi,
                      ") is not divisible by the world size ", world_);
          len /= world_;
          if (u.kind == ddl::RunnerUnit::RS) need_shard = std::max(need_shard, len);
        }
        need_state = std::max(need_state, range.state_off + len);
        u.ranges.push_back(range);
      }
      u.m = opt_ptr(t[5], need_state, "m");
      u.v = opt_ptr(t[6], need_state, "v");
      u.shard = opt_ptr(t[7], need_shard, "shard");
      out.push_back(std::move(u));
    }
    r_->set_units(out);
  }
  void set_optimizer(int64_t kind, double lr, double b1, double b2, double eps, double mu) {
    r_->set_optimizer((int)kind, (float)lr, (float)b1, (float)b2, (float)eps, (float)mu);
  }
  void set_scale(double grad_scale, double coef) { r_->set_scale((float)grad_scale, (float)coef); }
  void set_local_on_main(bool on) { r_->set_local_on_main(on); }
  void set_last_on_main(bool on) { r_->set_last_on_main(on); }
  void set_ready_flags(int64_t mode) { r_->set_ready_flags((int)mode); }
  void set_use_tail(bool on) { r_->set_use_tail(on); }
  void set_final_in_reduce(bool on) { r_->set_final_in_reduce(on); }
  void set_tail_cfg(int64_t first, int64_t f4) { r_->set_tail_cfg((int)first, (int)f4); }
  void step(at::Tensor x, at::Tensor labels, int64_t seed, std::vector<double> lr_t) {
    eng_.check_batch(x);
    TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_cuda(), "labels must be int64 GPU");
    TORCH_CHECK(labels.numel() == x.size(0), "labels/batch size mismatch");
    lr_.assign(lr_t.begin(), lr_t.end());
    if (lr_.empty()) lr_.push_back(0.f);
    r_->step(x.data_ptr<float>(), labels.data_ptr<int64_t>(), (int)x.size(0),
             (uint32_t)(seed & 0xFFFFFFFF), lr_.data(), cur_stream());
  }
  std::string async_error() { return r_->async_error(); }
  void abort() { r_->abort(); }
  void close() {
    py::gil_scoped_release nogil;
    r_->close();
  }
  py::tuple selftest() {
    std::string why;
    bool ok;
    {
      py::gil_scoped_release nogil;
      ok = r_->selftest(&why);
    }
    return py::make_tuple(ok, why);
  }

 private:
  PyEngine& eng_;
  at::Tensor params_, grads_;
  std::vector<at::Tensor> keep_;
  std::vector<float> lr_;
  std::unique_ptr<ddl::SyncRunner> r_;
  int64_t world_;
  PyPeer* peer_keep_ = nullptr;
};

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "ddl_amd native extension: gfx950 HIP kernels + C++ runtime";
  m.def("adam_flat", &adam_flat, "Fused TF1 Adam on a flat shard",
        py::arg("w"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("lr_t"), py::arg("b1"),
        py::arg("b2"), py::arg("eps"), py::arg("scale") = 1.0);
  m.def("momentum_flat", &momentum_flat, "Fused momentum SGD on a flat shard");
  // per-block timestamps of the split-K dual launches (kernels/stamps.h; a build with
  // DDL_STAMPS=1 records them, the default build records nothing)
  m.def("stamps_enabled", []() { return (bool)DDL_STAMPS; });
  m.def("stamps_begin", [](int64_t cap) {
    ddl::StampState& s = ddl::stamp_state();
    if (s.buf) (void)hipFree(s.buf);
    s.buf = nullptr;
    s.cap = s.next = 0;
    s.log.clear();
    if (cap <= 0) return;
    TORCH_CHECK(hipMalloc(&s.buf, (size_t)cap * 64) == hipSuccess, "stamp buffer");
    TORCH_CHECK(hipMemset(s.buf, 0, (size_t)cap * 64) == hipSuccess, "stamp buffer");
    s.cap = cap;
  });
  m.def("stamps_end", []() {
    ddl::StampState& s = ddl::stamp_state();
    TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "stamps: device sync");
    at::Tensor out = at::empty({(int64_t)s.next, 8}, at::kLong);
    if (s.next)
      TORCH_CHECK(hipMemcpy(out.data_ptr(), s.buf, (size_t)s.next * 64, hipMemcpyDeviceToHost) ==
                      hipSuccess, "stamps: copy");
    std::vector<std::vector<int64_t>> log;
    for (const auto& r : s.log) log.push_back({r.off, r.nblocks, r.sub, r.gx, r.gy, r.gz});
    if (s.buf) (void)hipFree(s.buf);
    s.buf = nullptr;
    s.cap = s.next = 0;
    s.log.clear();
    return std::make_pair(out, log);
  });
  m.def("mfma_peak", [](at::Tensor out, int64_t blocks, int64_t iters, int64_t kind) {
    check_f32_cuda(out, "out");
    TORCH_CHECK(out.numel() >= blocks * 64, "out too small");
    ddl::launch_mfma_peak(out.data_ptr<float>(), (int)blocks, (int)iters, cur_stream(), (int)kind);
  }, "diagnostic: per iteration 2 chains of v_mfma_f32_32x32x2_f32 (kind 0) or 4 of "
     "v_mfma_f32_16x16x4_f32 (kind 1), the same FLOPs", py::arg("out"), py::arg("blocks"),
     py::arg("iters"), py::arg("kind") = 0);
  m.def("gemm_nomem", [](at::Tensor out, at::Tensor slab, int64_t M, int64_t N, int64_t K,
                         int64_t splits) {
    ddl::launch_gemm_nomem(out.data_ptr<float>(), (int)M, (int)N, (int)K, (int)splits,
                           slab.data_ptr(), nullptr, cur_stream());
  }, "diagnostic: engine GEMM structure with register-only operand loads");
  m.def("xcd_sweep", [](at::Tensor a, c10::optional<at::Tensor> want, at::Tensor out) {
    check_f32_cuda(a, "a");
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kInt && out.numel() >= 2, "out: 2 int32");
    if (want) {
      check_f32_cuda(*want, "want");
      TORCH_CHECK(want->numel() == a.numel(), "want: same size as a");
    }
    ddl::launch_xcd_sweep(a.data_ptr<float>(), want ? want->data_ptr<float>() : nullptr,
                          a.numel(), out.data_ptr<int>(), cur_stream());
  }, "xGMI self-test probe: every XCD reads (warms) every line of a, or counts mismatches "
     "against want into out[0]", py::arg("a"), py::arg("want"), py::arg("out"));
  m.attr("OP_COUNT") = (int)ddl::OP_COUNT;

  py::class_<PyEngine>(m, "Engine")
      .def(py::init<std::vector<at::Tensor>, std::vector<at::Tensor>, int64_t, int64_t, double>(),
           py::arg("params"), py::arg("grads"), py::arg("max_batch"), py::arg("train_batch"),
           py::arg("keep_prob"))
      .def("set_keep_prob", &PyEngine::set_keep_prob)
      .def("set_splits", &PyEngine::set_splits)
      .def("get_splits", &PyEngine::get_splits)
      .def("set_cfg", &PyEngine::set_cfg)
      .def("get_cfg", &PyEngine::get_cfg)
      .def("set_eval_cfg", &PyEngine::set_eval_cfg)
      .def("get_eval_cfg", &PyEngine::get_eval_cfg)
      .def("set_concurrent", &PyEngine::set_concurrent)
      .def("set_dual", &PyEngine::set_dual)
      .def("set_conv1_direct", [](PyEngine& e, bool on) { e.raw()->conv1_direct = on; })
      .def("conv1_direct", [](PyEngine& e) { return e.raw()->conv1_direct; })
      .def("set_conv1_wgrad_direct", [](PyEngine& e, bool on) { e.raw()->conv1_wgrad_direct = on; })
      .def("conv1_wgrad_direct", [](PyEngine& e) { return e.raw()->conv1_wgrad_direct; })
      .def("set_wide_thr", &PyEngine::set_wide_thr)
      .def("set_wide", &PyEngine::set_wide)
      .def("set_dual_bfirst", &PyEngine::set_dual_bfirst)
      .def("get_dual_bfirst", &PyEngine::get_dual_bfirst)
      .def("get_wide", &PyEngine::get_wide)
      .def("forward", &PyEngine::forward, py::arg("x"), py::arg("seed"), py::arg("train"))
      .def("backward_segment", &PyEngine::backward_segment)
      .def("run_op", &PyEngine::run_op)
      .def("zero_correct", &PyEngine::zero_correct)
      .def("eval_count", &PyEngine::eval_count)
      .def("head_fwd", &PyEngine::head_fwd)
      .def("buffer", &PyEngine::buffer)
      .def("max_batch", &PyEngine::max_batch)
      .def("workspace_bytes", &PyEngine::workspace_bytes)
      .def_static("op_shape", &PyEngine::op_shape);

  py::class_<PyRunner>(m, "SyncRunner")
      .def(py::init<PyEngine&, at::Tensor, at::Tensor, int64_t, int64_t>(), py::arg("engine"),
           py::arg("params"), py::arg("grads"), py::arg("world"), py::arg("rank"),
           py::keep_alive<1, 2>())
      .def_static("unique_id", &PyRunner::unique_id)
      .def_static("probe", &PyRunner::probe)
      .def("init_comm", &PyRunner::init_comm, py::arg("id"), py::arg("force") = false)
      .def("has_comm", &PyRunner::has_comm)
      .def("set_units", &PyRunner::set_units)
      .def("set_optimizer", &PyRunner::set_optimizer)
      .def("set_scale", &PyRunner::set_scale)
      .def("set_local_on_main", &PyRunner::set_local_on_main)
      .def("set_last_on_main", &PyRunner::set_last_on_main)
      .def("set_use_tail", &PyRunner::set_use_tail)
      .def("set_ready_flags", &PyRunner::set_ready_flags)
      .def("set_final_in_reduce", &PyRunner::set_final_in_reduce)
      .def("set_tail_cfg", &PyRunner::set_tail_cfg)
      .def("step", &PyRunner::step)
      .def("selftest", &PyRunner::selftest)
      .def("set_peer", &PyRunner::set_peer, py::keep_alive<1, 2>())
      .def("peer_selftest_step", &PyRunner::peer_selftest_step)
      .def("async_error", &PyRunner::async_error)
      .def("abort", &PyRunner::abort)
      .def("close", &PyRunner::close);

  py::class_<PyAsyncPeer>(m, "AsyncPeer")
      .def(py::init<at::Tensor, at::Tensor, int64_t, int64_t, py::list, std::vector<int64_t>,
                    int64_t>(),
           py::arg("params"), py::arg("grads"), py::arg("world"), py::arg("rank"),
           py::arg("ranges"), py::arg("hosts"), py::arg("max_slices") = 512)
      .def("handle", &PyAsyncPeer::handle)
      .def("open", &PyAsyncPeer::open)
      .def("push_all", &PyAsyncPeer::push_all)
      .def("attach_done", &PyAsyncPeer::attach_done)
      .def("wait_done", &PyAsyncPeer::wait_done)
      .def("apply", &PyAsyncPeer::apply)
      .def("close", &PyAsyncPeer::close)
      .def("error", &PyAsyncPeer::error);

  py::class_<PyAsyncService>(m, "AsyncService")
      .def(py::init<PyAsyncPeer&, int64_t, py::list, int64_t, double, double, double,
                    double, double, double, int64_t, bool>(),
           py::keep_alive<1, 2>())
      .def("start", &PyAsyncService::start)
      .def("join", &PyAsyncService::join)
      .def("t", &PyAsyncService::t)
      .def("pause", &PyAsyncService::pause)
      .def("resume", &PyAsyncService::resume)
      .def("served", &PyAsyncService::served)
      .def("provenance", &PyAsyncService::provenance)
      .def("mode", &PyAsyncService::mode);

  py::class_<PyRcclAsync>(m, "RcclAsync")
      .def(py::init<at::Tensor, at::Tensor, int64_t, int64_t, py::list, std::vector<int64_t>,
                    py::list, int64_t, double, double, double, double, double, bool>())
      .def("init_comm", &PyRcclAsync::init_comm)
      .def("attach_shm", &PyRcclAsync::attach_shm)
      .def("open_boxes", &PyRcclAsync::open_boxes)
      .def("start", &PyRcclAsync::start)
      .def("push_pull", &PyRcclAsync::push_pull)
      .def("join", &PyRcclAsync::join)
      .def("pause", &PyRcclAsync::pause)
      .def("resume", &PyRcclAsync::resume)
      .def("t", &PyRcclAsync::t)
      .def("set_t", &PyRcclAsync::set_t)
      .def("served", &PyRcclAsync::served)
      .def("provenance", &PyRcclAsync::provenance);

  py::class_<PyAsyncRunner>(m, "AsyncRunner")
      .def(py::init<PyEngine&, PyAsyncPeer&, int64_t, int64_t, std::vector<int64_t>, int64_t>(),
           py::arg("engine"), py::arg("peer"), py::arg("world"), py::arg("rank"),
           py::arg("seg_of_ps"), py::arg("epoch0"),
           py::keep_alive<1, 2>(), py::keep_alive<1, 3>())
      .def("step", &PyAsyncRunner::step)
      .def("finish", &PyAsyncRunner::finish)
      .def("epoch", &PyAsyncRunner::epoch)
      .def("set_use_tail", &PyAsyncRunner::set_use_tail)
      .def("set_gate", &PyAsyncRunner::set_gate)
      .def("set_inline", &PyAsyncRunner::set_inline)
      .def("inline_on", &PyAsyncRunner::inline_on)
      .def("inline_t", &PyAsyncRunner::inline_t)
      .def("inline_sync_ps", &PyAsyncRunner::inline_sync_ps)
      .def("inline_provenance", &PyAsyncRunner::inline_provenance);

  py::class_<PyPeer>(m, "PeerExchange")
      .def(py::init<at::Tensor, at::Tensor, int64_t, int64_t, py::list, int64_t, int64_t>(),
           py::arg("params"), py::arg("grads"), py::arg("world"), py::arg("rank"),
           py::arg("buckets"), py::arg("max_slices") = 128, py::arg("repl_bucket") = -1)
      .def("handle", &PyPeer::handle)
      .def("open", &PyPeer::open)
      .def("error", &PyPeer::error)
      .def("nslices", &PyPeer::nslices)
      .def("owner", &PyPeer::owner)
      .def("close", &PyPeer::close);

  py::class_<ddl::ShmMailbox>(m, "ShmMailbox")
      .def(py::init<const std::string&, int64_t, bool>(), py::arg("name"), py::arg("capacity"),
           py::arg("create"))
      .def("push", &ddl::ShmMailbox::push, py::call_guard<py::gil_scoped_release>())
      .def("pop", &ddl::ShmMailbox::pop, py::call_guard<py::gil_scoped_release>())
      .def("size", &ddl::ShmMailbox::size)
      .def("capacity", &ddl::ShmMailbox::capacity)
      .def("unlink", &ddl::ShmMailbox::unlink);
}
