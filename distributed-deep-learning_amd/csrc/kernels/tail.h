// Optimizer "tail" riding in a GEMM launch (host-visible descriptor; device body in gemm.h).
//
// With one worker (W = 1) every PS update is local and the step is one packed queue, so a
// stand-alone Adam launch at the end of the step is pure critical path: an HBM-bound pass
// over w, g, m, v (≈74 MB for the 2.66 M parameters, 18.5 us measured) after the last
// backward GEMM.  A segment's gradients are final once its backward launches have run, and
// no later backward launch reads that segment's parameters, so the update of segment s can
// run as extra blocks of segment s+1's dual dgrad+wgrad launch: memory-bound blocks beside
// MFMA-bound ones, hidden instead of serialised.  Only the last segment's (conv1 + conv2,
// 52 k parameters) update remains a launch of its own.
//
// The asynchronous worker step (async_runner.hip) uses the same slot for its gradient PUSH
// (kind 1): segment s's shards are stored into their PS hosts' inboxes and posted on the
// arrival board by tail blocks of segment s+1's first launch instead of a push kernel of their
// own on the compute stream (~5 us each, latency-bound).  One block per arrival slice.
//
// Kind 2 is a READY flag: the synchronous runner's xGMI bucket kernels on the comm stream wait
// (behind a one-wave gate there) for segment s's gradients; block 0 of the tail stores
// p[0].arrive[0] = epoch at the start of segment s+1's first launch, which the stream starts only
// after every launch of segment s has completed.  It replaces an event record / stream wait
// pair (~5 us of idle compute stream each, runner.hip).
#pragma once
#include <stdint.h>

namespace ddl {

constexpr int kTailPieces = 4;
constexpr int kTailF4PerLane = 2;  // float4 per lane per pass: keeps the tail path under the GEMM paths' VGPRs
constexpr int kTailF4PerBlock = 64 * kTailF4PerLane;  // one-wave blocks
// float4 per tail block of a segment's Adam riding beside a dual launch's GEMM blocks (8 passes
// of one wave; round 6, scripts/sched_ab.py --tail-variants: 256 / 512 / 768 / 1024 / 1280 /
// 1536 / 2048 float4: 263.6 / 262.3-262.9 / 261.5 / 260.8-261.5 / 261.5 / 264.1 / 271.4 us/step,
// profiles/r6_sched_ab_tail.log)
constexpr int kTailF4Default = 8 * kTailF4PerBlock;

struct UpdPiece {
  float* w = nullptr;      // 16-B aligned, n % 4 == 0 (checked by the host); push: the inbox slot
  const float* g = nullptr;  // push: the gradient shard
  float* m = nullptr;
  float* v = nullptr;
  int64_t n = 0;           // elements
  float lr_t = 0.f;        // TF1 Adam step size of the owning PS
  int blk0 = 0;            // first tail block of this piece
  // push (kind 1): slice j = block blk0 + j covers float4 [j * slice4, (j + 1) * slice4); its
  // board word posted[j] (host memory).  Ready flag
  // (kind 2): arrive[0]
  uint32_t* arrive = nullptr;
  uint32_t* posted = nullptr;
  int slice4 = 0, nslice = 0;
};

struct UpdTail {
  int nblocks = 0;         // tail blocks (multiple of 8: keeps the GEMM blocks' XCD mapping)
  int npieces = 0;
  int kind = 0;            // 0: Adam update, 1: asynchronous gradient push (round `epoch`),
                           // 2: ready flag (p[0].arrive[0] = epoch)
  uint32_t epoch = 0;
  int first = 1;           // 1: tail blocks precede the GEMM blocks in the grid, 0: follow them
  int f4_per_block = kTailF4PerBlock;  // float4 per tail block (multiple of kTailF4PerBlock)
  UpdPiece p[kTailPieces];
  float c1 = 0.f, c2 = 0.f, eps = 0.f, scale = 1.f;  // 1 - beta1, 1 - beta2, epsilon, grad scale
};

}  // namespace ddl
