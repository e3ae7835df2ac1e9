/*
 * sfx.h -- C ABI of libsfx.so, the MI355X (gfx950) successor-feature hot path.
 *
 * The reference (okgarces/deep-successor-features-for-transfer) is pure Python; its
 * plugin surface for this path is the duck-typed SF object (features/successor.py:6-290,
 * features/deep.py, sfdqn.py:94-371).  Each entry point below replaces the reference
 * call cited next to it; the Python layer (deep-successor-features-for-transfer_amd/sfx)
 * binds these with ctypes exactly as INTEGRATION.md shows.
 *
 * Conventions
 *  - Every pointer argument named *_dev is a DEVICE pointer (hipMalloc / torch CUDA
 *    tensor), read/written asynchronously on the handle's stream.  Host pointers are
 *    named *_host and are read/written synchronously.
 *  - All floating point data is fp32.  Actions and argmax indices are int64 (torch.long).
 *  - A ψ head is packed as the reference's nn.Sequential parameters() in order:
 *    for each Linear, weight[out][in] row-major then bias[out] ("torch packing").
 *    Internally each tensor starts 16-byte aligned; load/get convert.
 *  - Return value: 0 on success, a negative SFX_E* code otherwise; sfx_last_error()
 *    returns a message.  The Python layer raises on any non-zero status.
 *  - One handle = one device; calls are not thread-safe on the same handle.
 */
#ifndef SFX_H
#define SFX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SFX_OK 0
#define SFX_E_ARG (-1)
#define SFX_E_HIP (-2)
#define SFX_E_STATE (-3)

#define SFX_ACT_NONE 0
#define SFX_ACT_RELU 1
#define SFX_ACT_TANH 2

#define SFX_PREC_FP32 0 /* the reference's arithmetic; every parity test runs in it (default) */
#define SFX_PREC_BF16 1 /* bf16 MFMA operands for the forward and dX GEMMs, fp32 elsewhere */

typedef struct sfx_handle* sfx_t;

/* Version string of the build (for logs). */
const char* sfx_version(void);
/* Message describing the last failure on this thread. */
const char* sfx_last_error(void);
/* Device bounds checks of the check build (libsfx_check.so, -DSFX_CHECK): the number of
 * failed checks since the last reset (count = -1 in the product build); first_host: up to 8
 * records of (source line, a, b, c) or null; reset != 0 clears the count. */
int sfx_check_failures(long long* count, long long* first_host, int reset);

/*
 * Create the per-device library state for T ψ heads of geometry
 *   Linear(n_s,H) -> [Linear(H,H)+act_i for i < n_hidden] -> Linear(H, A*d)
 * (the lambda of main_sfdqn_torch.py:44-78, built per task by DeepSF.build_successor,
 * features/deep.py:39-78 / sfdqn.py:242-288).  max_batch bounds the minibatch rows of
 * one update (reference buffer n_batch=32, configs/reacher.cfg:265-267).
 * stream: hipStream_t the handle launches on (NULL = legacy default stream).
 */
int sfx_create(sfx_t* out, int T, int n_s, int H, int n_hidden, const int* acts_host, int A,
               int d, int max_batch, int device, void* stream);
int sfx_destroy(sfx_t h);
int sfx_set_stream(sfx_t h, void* stream);
/* Each entry point's launch sequence is captured into a hipGraph keyed by its arguments
 * and replayed on later calls with the same arguments (default on; SFX_GRAPHS=0 in the
 * environment or enable=0 here launches eagerly). */
int sfx_set_graphs(sfx_t h, int enable);
/* Packed parameter count of one head in torch packing. */
int sfx_head_numel(sfx_t h);

/*
 * Adam hyper-parameters (torch.optim.Adam single-tensor semantics,
 * torch/optim/adam.py:_single_tensor_adam) for the ψ group and the w group
 * (sfdqn.py:282-286: {'lr': learning_rate_sf, 'weight_decay': weight_decay_sf},
 *  {'lr': learning_rate_w, 'weight_decay': weight_decay_w}).
 */
int sfx_set_adam(sfx_t h, double lr_psi, double wd_psi, double lr_w, double wd_w, double beta1,
                 double beta2, double eps);

/* Parameter I/O (replaces building / reading the per-task nn.Sequential:
 * features/deep.py:50-66, utils/torch.py:31-33).  which: 0 online, 1 target. */
int sfx_load_head(sfx_t h, int t, int which, const float* params_host);
int sfx_get_head(sfx_t h, int t, int which, float* params_host);
/* Adam state of head t: m, v in torch packing; step = optimizer step count. */
int sfx_load_adam(sfx_t h, int t, const float* m_host, const float* v_host, int step);
int sfx_get_adam(sfx_t h, int t, float* m_host, float* v_host, int* step);
/* Reward weights w_t (d floats): fit_w of SF.add_training_task (features/successor.py:134-139)
 * or the Linear(d,1,bias=False) weight of sfdqn.py:196-204. */
int sfx_load_w(sfx_t h, int t, const float* w_host);
int sfx_get_w(sfx_t h, int t, float* w_host, float* wm_host, float* wv_host);
/* w_t and its Adam moments (sfdqn.py:196-204's w optimizer state), e.g. to resume from a
 * checkpoint (sfx/checkpoint.py). */
int sfx_load_w_state(sfx_t h, int t, const float* w_host, const float* wm_host, const float* wv_host);
/* Device pointer to w row t (d floats), stable for the handle's lifetime. */
int sfx_w_ptr(sfx_t h, int t, float** w_dev);

/*
 * GPI over all heads (SF.GPI_w, features/successor.py:223-246; sfdqn.py:215-240;
 * DeepSF.get_successors, features/deep.py:85-91):
 *   psi[b,t,:,:] = ψ_t(S[b]);  q[b,t,a] = ψ[b,t,a,:]·w;
 *   task[b] = argmax_t max_a q[b,t,a];  next[b] = argmax_a max_t q[b,t,a]
 * (first index on ties, as torch.argmax).  S_dev [B, n_s], w_dev [d].  Any output
 * pointer may be NULL.  psi_dev [B,T,A,d], q_dev [B,T,A], task_dev/next_dev [B].
 */
int sfx_gpi(sfx_t h, const float* S_dev, int B, const float* w_dev, float* psi_dev, float* q_dev,
            int64_t* task_dev, int64_t* next_dev);

/*
 * Successor features of every head, online (which = 0: DeepSF.get_successors,
 * features/deep.py:85-91; features/deep_sequential_tsf.py:150-158) or target (which = 1:
 * DeepTSF.get_next_successors, features/deep_sequential_tsf.py:160-174; tsfdqn.py:296-307):
 * psi_dev[b,t,:,:] = ψ_t(S[b]) (ψ⁻_t for which = 1), [B,T,A,d].
 */
int sfx_successors(sfx_t h, const float* S_dev, int B, int which, float* psi_dev);

/*
 * Greedy action of Agent.next_sample for one encoded state (sfdqn.py:585-594;
 * agents/sfdqn.py:39-45 + agents/agent.py:144-157 greedy branch):
 *   (q, c) = GPI(s, task_index); c = task_index unless use_gpi; a = argmax_a q[0,c,:].
 * out_dev[0] = c (GPI task), out_dev[1] = a.  q_dev [T, A] may be NULL.
 */
int sfx_select_action(sfx_t h, const float* s_dev, int task_index, int use_gpi, float* q_dev,
                      int64_t* out_dev);

/*
 * Greedy test-task actions of E test tasks at once, each with its own reward weights
 * (SFDQN.get_test_action's greedy branch, agents/sfdqn.py:125-137, for every test task of one
 * lockstep step of agents/sfdqn.py:111-115 / test_agent :139-166):
 *   q[e,t,a] = ψ_t(S[e])[a,:]·W[e,:];  c_e = argmax_t max_a q[e,t,a];  a_e = argmax_a q[e,c_e,a]
 * (first index on ties).  S_dev [E, n_s], W_dev rows w_stride >= d floats apart,
 * out_dev [E, 2] = (c_e, a_e), q_dev [E, T, A] may be NULL.
 */
int sfx_test_actions(sfx_t h, const float* S_dev, int E, const float* W_dev, int w_stride, float* q_dev,
                     int64_t* out_dev);

/*
 * The test tasks' reward models of one lockstep step: SFDQN.update_test_reward_mapper
 * (agents/sfdqn.py:168-184: a fresh SGD(lr=0.005, weight_decay=0.01) step on the bias-free
 * Linear(d, 1) w_e, loss MSE(w_e(φ_e), r_e)) for E test tasks in one launch.  phi_dev [E, d]
 * contiguous, r_dev [E], W_dev rows w_stride >= d floats apart (updated in place), loss_dev [E]
 * = the pre-step losses the reference returns.  Asynchronous on the handle's stream.
 */
int sfx_test_reward_updates(sfx_t h, int E, const float* phi_dev, const float* r_dev, float* W_dev, int w_stride,
                            double lr, double wd, float* loss_dev);

/*
 * One SF TD update of head `policy` (DeepSF.update_successor, sfdqn.py:303-371 ==
 * features/deep_sequential.py:163-231): GPI (or own-ψ) next actions over S1, targets
 * φ + γ ψ⁻_i(S1)[a'], l1 = MSE(ψ_i(S), merged) [+ l2 = MSE(w_i·φ, r) when r_dev != NULL,
 * which also trains w_i], one Adam step, target sync every target_update_ev updates.
 * Inputs: S, S1 [B, n_s]; a [B] int64; r [B] (or NULL); phi [B, d]; gamma [B].
 * losses_dev[3] = (l1 + l2, l1, l2) (may be NULL); next_dev [B] (may be NULL).
 */
int sfx_update(sfx_t h, int policy, const float* S_dev, const int64_t* a_dev, const float* r_dev,
               const float* phi_dev, const float* S1_dev, const float* gamma_dev, int B,
               int use_gpi, float* losses_dev, int64_t* next_dev);

/*
 * All-task update (agents/sfdqn.py:57-60 looping features/deep.py:93-131 over every
 * head in index order, each GPI seeing the heads already updated in this call).
 * loss = l1 only, w_i not trained (LMS w).  losses_dev [T, 3] (may be NULL).
 * Returns once the step is enqueued on the handle's stream: the speculation verdict (and host
 * rounds, should the device rounds leave a policy unverified) is collected by the next call on
 * the handle -- every entry point does that first -- so losses_dev is complete in stream order and
 * any result read through the API reflects the whole update.
 */
int sfx_update_all(sfx_t h, const float* S_dev, const int64_t* a_dev, const float* phi_dev,
                   const float* S1_dev, const float* gamma_dev, int B, float* losses_dev);

/*
 * One env step's library work of the all-task agent in one launch set: the LMS reward fit of
 * w[lms_task] on (lms_phi [d], r) when lms_task >= 0 (SF.update_reward, features/
 * successor.py:164-167; r = *lms_r_dev when lms_r_dev != NULL -- the reference's tasks return the
 * reward as a device tensor -- else the value lms_r), sfx_update_all,
 * then the agent loop's next GPI (agents/agent.py:223-224 -> agents/sfdqn.py:39-45 ->
 * features/successor.py:248-273) when its state is already known: the transition's next state
 * s_next_dev [n_s] with w[task_index].  q_dev [T * A] and task_dev [1] (device, may be NULL)
 * receive what sfx_lms + sfx_update_all + sfx_gpi(h, s_next, 1, w[task_index], NULL, q, task,
 * NULL) write, bit for bit; the LMS rides in the step's first launch and the selection in its
 * final round (and again in any host round).  Like sfx_update_all it returns once enqueued;
 * sfx_settle (or any later call) collects the verdict.
 */
int sfx_update_all_select(sfx_t h, const float* S_dev, const int64_t* a_dev, const float* phi_dev,
                          const float* S1_dev, const float* gamma_dev, int B, float* losses_dev,
                          const float* s_next_dev, int task_index, float* q_dev, int64_t* task_dev, int lms_task,
                          const float* lms_phi_dev, float lms_r, const float* lms_r_dev, float lms_alpha);
/* Collect the verdict of a pending sfx_update_all / sfx_update_all_select (waits for the step;
 * host rounds when the device rounds left a policy unverified).  A no-op without one.
 * host_rounds (may be NULL): the rounds this call ran on the host (0 when the device rounds held;
 * sfx_update_all_select's q / task were then rewritten after the host rounds).  sel (may be NULL):
 * [2] the collected step's selection (GPI task c, greedy action) -- c is the task sfx_update_all_select
 * wrote -- or -1 when this call collected no step with a selection. */
int sfx_settle(sfx_t h, int* host_rounds, int64_t* sel);

/*
 * Fused env step of the all-task schedule: the device half of one Agent.next_sample
 * (agents/agent.py:195-261) with SFDQN.train_agent (agents/sfdqn.py:47-60):
 *   - LMS reward fit of w[lms_task] on (lms_phi [d], lms_r [1]) when lms_task >= 0
 *     (SF.update_reward, features/successor.py:164-167);
 *   - when B > 0, every head updated on the minibatch exactly as the reference's in-order
 *     loop does.  The update is launched SPECULATIVELY (all policies take their GPI next
 *     actions from the pre-step heads, the heads update in parallel into their second
 *     parameter slot); the device then re-derives each policy's next actions with the
 *     heads before it already updated and flags the first policy whose actions differ;
 *   - when s_next != NULL, the GPI greedy action for s_next with w[task_index] on the
 *     updated heads (sfdqn.py:585-594).
 * sfx_step_all only launches; sfx_step_finish waits, runs further rounds while a policy is
 * flagged (each round makes at least one more head exact), commits, and writes
 * out_host[0] = GPI task c, [1] = greedy action, [2] = first policy flagged by the last
 * device round (T when it held).  losses_dev [T, 3] may be NULL.
 */
int sfx_step_all(sfx_t h, const float* S_dev, const int64_t* a_dev, const float* phi_dev, const float* S1_dev,
                 const float* gamma_dev, int B, int use_gpi, int lms_task, const float* lms_phi_dev,
                 const float* lms_r_dev, float lms_alpha, const float* s_next_dev, int task_index, int sel_use_gpi,
                 float* losses_dev);
int sfx_step_finish(sfx_t h, int64_t* out_host);
/* Test hook: make every following fused step run one more round as if the speculation had
 * failed at first_policy (-1: off).  Results must not change. */
int sfx_debug_force_rerun(sfx_t h, int first_policy);
/* Speculative rounds launched on the device per fused step; 0 = automatic (the default): 2 for
 * fewer than 16 source tasks (T_glob, after sfx_shard_setup), 3 from 16 on.  Round r > 0
 * re-derives every policy's next actions from round r-1's updated heads; a step whose
 * last device round still flags a policy gets further rounds from sfx_step_finish. */
int sfx_set_spec_rounds(sfx_t h, int rounds);
/* Operand precision of the ψ GEMMs (north_star: "MFMA bf16 for the small dense MLP GEMMs").
 * SFX_PREC_BF16: the forward and dX tiles take bf16 operands (v_mfma_f32_16x16x32_bf16) from
 * bf16 copies of the online / target parameters, accumulate in fp32; the master parameters,
 * Adam moments, dW, TD target, GPI, losses stay fp32, and the Adam epilogue refreshes the copy
 * of every parameter it writes.  Not bit-exact with the reference (argmax agrees
 * wherever the top-2 gap exceeds the bf16 error).  Default SFX_PREC_FP32. */
int sfx_set_precision(sfx_t h, int precision);
int sfx_get_precision(sfx_t h);
/* The ψ loss (sfdqn.py:341-342 and every update path that shares its TD kernels: the all-task
 * step, sfx_update, TSF, learned φ, sharded heads).  delta == 0 (default): MSELoss(mean), the
 * reference's.  delta > 0: opt-in HuberLoss(delta, mean) -- north_star names a "Huber backward",
 * the reference has none, so this is an extra: gradient (1/N) clamp(c - t, -δ, δ) as
 * torch's huber_loss_backward forms it, losses 0.5 x² / δ(|x| - 0.5δ) per element.
 * delta < 0 or not finite: SFX_E_ARG.  sfx_get_huber returns the current delta. */
int sfx_set_huber(sfx_t h, float delta);
float sfx_get_huber(sfx_t h);
/* Counters of fused steps: total, those that needed host-issued rounds, the policies
 * still unverified after the device rounds, and all rounds run. */
int sfx_step_stats(sfx_t h, long long* steps, long long* fallbacks, long long* rerun_policies, long long* rounds);
/* Speculative rounds r >= 1 skip a policy whose next actions repeat round r-1's (its update
 * would repeat bit for bit): policies checked and skipped so far, counted on the device
 * (synchronises the handle's stream); reset != 0 zeroes the counters afterwards. */
int sfx_skip_stats(sfx_t h, long long* checked, long long* skipped, int reset);
/* Launch-graph cache of the handle: graphs captured (and instantiated) so far, graph launches,
 * graphs currently cached.  A call whose device pointers or configuration the cache has not seen
 * captures a new graph; a steady loop should capture only while it warms up. */
int sfx_graph_stats(sfx_t h, long long* captures, long long* launches, long long* cached);

/*
 * Failure detection (the reference only prints NaN/Inf diagnostics,
 * features/deep_phi.py:185-192): every TD-target kernel sets a sticky device flag when a TD error
 * c - (φ + γ ψ⁻) comes out non-finite (NaN or Inf in φ, γ, the ψ heads or the target heads).  The
 * native runner publishes the flag with each step's result and fails the run at the first such
 * step; sfx_nonfinite reads it (flag_host = 0 / 1) and optionally resets it.
 */
int sfx_nonfinite(sfx_t h, int* flag_host, int reset);

/*
 * The drop-in's agents.buffer ring (replaces agents/buffer.py:62-82 append and :34-60 replay's
 * collation): device arrays rs [cap][n_s], rphi [cap][d], rs1 [cap][n_s], ra [cap] (int64).
 * sfx_replay_put writes row j from device vectors s, phi, s1 and the int64 scalar *a in one
 * launch; sfx_replay_gather writes the minibatch rows idx[0, B) (device int64) into S, PHI, S1, A
 * and the discount factors into G -- from rg [cap] when non-null, else gam [B] -- in one launch.
 * Both enqueue on `stream` (a hipStream_t; NULL = the legacy default stream) and need no handle.
 */
int sfx_replay_put(void* stream, float* rs, float* rphi, float* rs1, int64_t* ra, long long j, const float* s,
                   const float* phi, const float* s1, const int64_t* a, int n_s, int d);
/* sfx_replay_put of row j followed by sfx_replay_gather (rows idx[0, B); γ from rg, or gam when
 * rg is NULL) in ONE launch -- the append and the replay of agents/agent.py:251-256 -- a row idx[b]
 * == j read from the new transition itself.  s1_copy [n_s] / phi_copy [d] (may be NULL) receive
 * copies of s1 and phi: the drop-in hands the agent's next GPI state and the LMS features to the
 * fixed inputs of sfx_update_all_select this way (no launch of their own, graph keys that do not
 * change). */
int sfx_replay_put_gather(void* stream, float* rs, float* rphi, float* rs1, int64_t* ra, const float* rg, long long j,
                          const float* s, const float* phi, const float* s1, const int64_t* a, float* s1_copy,
                          float* phi_copy, const int64_t* idx, const float* gam, int B, float* S, float* PHI,
                          float* S1, int64_t* A, float* G, int n_s, int d);
int sfx_replay_gather(void* stream, const float* rs, const float* rphi, const float* rs1, const int64_t* ra,
                      const float* rg, const int64_t* idx, const float* gam, int B, float* S, float* PHI, float* S1,
                      int64_t* A, float* G, int n_s, int d);
/* Host memory the kernels read directly, coherently (hipHostMalloc coherent + mapped): the drop-in
 * replay hands the minibatch's indices and γ to sfx_replay_gather in it instead of copying them. */
int sfx_host_alloc(size_t bytes, void** out);
int sfx_host_free(void* p);

/* LMS reward fit SF.update_reward (features/successor.py:164-167) on w_t:
 * w <- w + alpha (r - φ·w) φ ;  phi_dev [d], r_dev [1]. */
int sfx_lms(sfx_t h, int t, const float* phi_dev, const float* r_dev, float alpha);
/* The same with the reward as a value (the reference's agents pass a host float; features/
 * successor.py:164-167): no host->device copy of r, one launch. */
int sfx_lms_value(sfx_t h, int t, const float* phi_dev, float r, float alpha);

/* Target bookkeeping (sfdqn.py:366-369; utils/torch.py:31-33). */
int sfx_set_target_update_ev(sfx_t h, int target_update_ev);
int sfx_get_since_target(sfx_t h, int t, int* count);
int sfx_set_since_target(sfx_t h, int t, int count);
int sfx_sync_target(sfx_t h, int t);

/*
 * Event instrumentation for the benchmark's roofline figure: while enabled, graphs are
 * bypassed and every kernel launch is bracketed by a hipEvent pair.  Kinds:
 * 0 forward, 1 TD target, 2 backward+Adam, 3 GPI, 4 LMS, 5 speculation check, 6 TSF transform
 * (k_tsf_fwd / k_tsf_bwd) and learned φ.  collect() returns the number of
 * launches of that kind, their summed event-measured duration (us) and their summed
 * ALGORITHMIC bytes (what the launch must read/write at minimum, fp32).
 */
#define SFX_K_FWD 0
#define SFX_K_TDG 1
#define SFX_K_BWD 2
#define SFX_K_GPI 3
#define SFX_K_LMS 4
#define SFX_K_VER 5
#define SFX_K_ROUND 6
#define SFX_K_TSF 7
int sfx_prof_enable(sfx_t h, int enable);
int sfx_prof_collect(sfx_t h, int kind, int* count, double* total_us, double* bytes);
int sfx_prof_reset(sfx_t h);

/* Block the host until all work queued on the handle's stream is done. */
int sfx_synchronize(sfx_t h);

/* ---------------------------------------------------------------------------------------
 * Native env-step runner (replaces the Python loop of Agent.next_sample + SFDQN.train_agent,
 * agents/agent.py:195-261 with agents/sfdqn.py:39-60, for the all-task schedule of
 * main_sfdqn_torch.py).  The env and the replay ring stay on the host; each env step's device
 * work is one pre-launched hipGraph whose first kernel waits for the host's inputs.
 * Env callbacks (both or neither; NULL = built-in synthetic Reacher-shape task: s ~ N(0,1),
 * φ ~ U[0,1), r = φ[task % d], never terminal):
 *   reset(ctx, task, s0_host[n_s]);  step(ctx, task, action, s1_host[n_s], phi_host[d],
 *   r_host[1], terminal_host[1]);  return 0 on success.
 * ------------------------------------------------------------------------------------- */
typedef struct sfx_runner* sfx_runner_t;
typedef int (*sfx_env_reset_fn)(void* ctx, int task, float* s0_host);
typedef int (*sfx_env_step_fn)(void* ctx, int task, int action, float* s1_host, float* phi_host,
                               float* r_host, int* terminal_host);

/* batch: minibatch rows (buffer n_batch); capacity: replay ring size; gamma: discount of
 * non-terminal transitions; epsilon: ε-greedy rate; alpha_w: LMS rate of update_reward;
 * episode_len: T of the env episode; sel_use_gpi: GPI (1) or own-task (0) action choice. */
int sfx_runner_create(sfx_runner_t* out, sfx_t h, int batch, int capacity, float gamma, float epsilon,
                      float alpha_w, int episode_len, int sel_use_gpi, unsigned long long seed,
                      sfx_env_reset_fn reset_fn, sfx_env_step_fn step_fn, void* env_ctx);
int sfx_runner_destroy(sfx_runner_t r);
/* byte offsets of one step's input record: s, s1, phi, a(int64), gamma, s_next, phi1, r1,
 * r (minibatch rewards [batch]), total */
int sfx_runner_layout(sfx_runner_t r, int64_t* offsets_host /* [10] */);
/* training schedule of the env steps: 0 all-task (default; agents/sfdqn.py:47-60 with LMS w),
 * 1 active task only (sfdqn.py:462-471, agents/sfdqn_sequential.py:63-76: l1 + l2, Adam w),
 * 2 TSF-DQN active task (tsfdqn.py:566-580; needs sfx_tsf_setup), 3 all-task with the heads
 * sharded over ranks (BASELINE config C4; needs sfx_shard_setup and a communicator), 4 TSF-DQN
 * active task with the heads sharded over ranks (config C5, tsfdqn_nf.py:598-612: the active
 * policy's GPI maxima all-reduced, its owner updates, h and w_task handed to every rank by libsfx
 * collectives; needs sfx_tsf_setup, sfx_shard_setup and a communicator; the active task of
 * sfx_runner_set_task is then a global index).  use_gpi: next actions of the
 * update by GPI (1) or the own head (0).  p_end: episode-end probability per step of the
 * built-in synthetic task (γ = 0 on that transition; 0 = never, like tasks/reacher.py:112).
 * Call between runs (before sfx_runner_set_task). */
int sfx_runner_config(sfx_runner_t r, int schedule, int use_gpi, float p_end);
/* Device-resident replay (opt-in -- the north_star keeps the replay on the
 * host, and so does the headline bench): the ring moves to HBM, each step hands the device only
 * its transition, and the step's gate kernel appends it and draws the uniform minibatch (index
 * function replay_index in csrc/sfx_kernels.h).  The host ring stays as a mirror (prefill,
 * records); switching uploads it before the next run.  Replaces agents/buffer.py:34-64. */
int sfx_runner_device_replay(sfx_runner_t r, int enable);
/* Agent.set_active_training_task (agents/agent.py:121-139): reset the env, select the first action */
int sfx_runner_set_task(sfx_runner_t r, int task);
/* n random transitions into the replay (warm-up; not env steps) */
int sfx_runner_prefill(sfx_runner_t r, int n);
/* n env steps; returns with every step finished */
int sfx_runner_run(sfx_runner_t r, int n);
/* [GPI task c, greedy action, active task] for the current state */
int sfx_runner_action(sfx_runner_t r, int64_t* out_host /* [3] */);
int sfx_runner_stats(sfx_runner_t r, long long* env_steps, long long* prelaunched, long long* host_round_steps,
                     double* wait_us);
/* Bound of a step's gate wait (default 5 s).  A step whose inputs the host releases later is
 * cancelled at its gate -- none of its launches commits parameters, moments, step counters or w --
 * and the runner issues it again from the same staged inputs (counted by sfx_runner_retried).
 * On any error of sfx_runner_run (an env callback, a launch, the device) the steps queued behind
 * the host are cancelled the same way before the error returns: the heads hold the last
 * completed step and the runner stays usable. */
int sfx_runner_gate_timeout(sfx_runner_t r, double seconds);
/* Bound of the host's wait on a step's published result (default 10 s).  Past it the runner
 * cancels the queued steps and drains the device queue (bounded); when the queue does not drain
 * -- a sharded step's collective waiting for a peer that is gone -- it reads RCCL's asynchronous
 * error (ncclCommGetAsyncError), aborts the handle's communicators (ncclCommAbort; a borrowed
 * sfx_set_comm communicator too) and returns SFX_E_STATE; every later collective of the handle
 * fails with that error, and a runner whose queue never drained fails every call. */
int sfx_runner_wait_timeout(sfx_runner_t r, double seconds);
/* While the host runs host rounds of a step (speculation not verified on the device), the next
 * step's gate does not give up (hold protocol) -- for at most max(bound, 20 s). */
/* Instantiate the step graphs of the current schedule and task ahead of the first steps (every
 * span length, both slot parities) without running them: a short run then measures replays, not
 * graph captures. */
int sfx_runner_warm(sfx_runner_t r);
/* Steps issued again after their gate gave up (the step in flight, or steps queued behind it). */
int sfx_runner_retried(sfx_runner_t r, long long* retried);
/* Look-ahead (all-task schedule with the host replay; SFX_AHEAD=0 turns it off): the final
 * speculative round of env step E also runs the forward of step E+1's minibatch -- its indices are
 * drawn a step early from the runner's own index stream -- into the other copy of the minibatch
 * activations, so step E+1 opens with its TD launch (its gate resets the speculation flag and runs
 * the LMS fit).  pre_steps: steps that started so; own_forward_steps: steps with an update that ran
 * their own forward (their minibatch sampled the slot of their own transition, whose next state
 * was unknown a step early; the first step of a run; after a target sync or a drain). */
int sfx_runner_ahead_stats(sfx_runner_t r, long long* pre_steps, long long* own_forward_steps);
/* Steps whose host rounds found later steps cancelled at their gates: those steps' launches ran
 * (committing nothing) over the transient buffers the rounds read, so the step's forward and
 * device rounds were recomputed from its pre-step slot first. */
int sfx_runner_recomputed(sfx_runner_t r, long long* recomputed);
/* Steps whose published result carried the non-finite TD flag (sfx_nonfinite); the runner returns
 * SFX_E_STATE at the first one. */
int sfx_runner_nonfinite(sfx_runner_t r, long long* steps);
/* SF.gpi_counters (features/successor.py:270-272): [T][T] counts of the GPI task per active task
 * (counted only with GPI action selection, as SF.GPI(update_counters=use_gpi), agents/sfdqn.py:41) */
int sfx_runner_gpi_counters(sfx_runner_t r, long long* out_host /* [T*T] */);
/* test hooks: keep the input record and (task, have_batch, c, greedy a, taken a, terminal) of
 * the next `capacity` steps */
int sfx_runner_record(sfx_runner_t r, int capacity);
int sfx_runner_recorded(sfx_runner_t r);
int sfx_runner_get_record(sfx_runner_t r, int i, void* stage_host, int64_t* meta_host /* [6] */);

/* ---------------------------------------------------------------------------------------
 * Collective of the sharded step (SURVEY.md §8b sfx_set_comm, §8e): all-reduce(MAX) of fp32
 * GPI maxima over the ranks that share the source tasks.  Replaces the reference's in-process
 * loop over all heads (agents/sfdqn.py:57-60 / SF.GPI, features/successor.py:223-273) when the
 * heads live on several GPUs.  One of:
 *  - sfx_comm_init: the library creates (and owns) an RCCL communicator from a unique id that
 *    rank 0 made with sfx_comm_unique_id and the caller distributed (e.g. over torch.distributed);
 *    all ranks call it together;
 *  - sfx_set_comm: the caller's ncclComm_t (borrowed; it must outlive the handle's use of it);
 *  - sfx_set_comm_host: a host callback all-reducing (MAX, in place) a pinned host buffer -- for
 *    ranks that cannot run RCCL (several ranks on one GPU in tests); its steps are not graphed.
 * RCCL all-reduces are enqueued on the handle's stream and captured into the step graphs.
 * ------------------------------------------------------------------------------------- */
/* GPI maxima cross ranks as "sortable" int32: the order-preserving map of the fp32 value
 * (i = bits(f + 0); i >= 0 ? i : i ^ 0x7FFFFFFF), so all-reduce(MAX) runs on int32 and the
 * decoded maximum is exactly the fp32 one; INT32_MIN marks an empty entry. */
typedef int (*sfx_host_allreduce_fn)(void* ctx, int32_t* buf_host, int count);
int sfx_comm_id_bytes(void);
int sfx_comm_unique_id(void* id_out /* sfx_comm_id_bytes() bytes */);
int sfx_comm_init(sfx_t h, const void* unique_id, int rank, int world);
int sfx_set_comm(sfx_t h, void* rccl_comm, int rank, int world);
int sfx_set_comm_host(sfx_t h, sfx_host_allreduce_fn fn, void* ctx, int rank, int world);
/* Communicator state: bit 0 step communicator, bit 1 the host rounds' communicator (split off by
 * sfx_comm_init / sfx_set_comm with ncclCommSplit; with it the runner pipelines sharded steps at
 * N > 1 too), bit 2 aborted after a timed-out collective, bit 3 host transport.  RCCL is loaded
 * at run time (dlopen) by the first RCCL call. */
int sfx_comm_state(sfx_t h, int* state);
/* Rank / world the handle was given, and what its RCCL communicator itself reports
 * (ncclCommUserRank / ncclCommCount; -1 / 0 without an RCCL communicator). */
int sfx_comm_size(sfx_t h, int* rank, int* world, int* rccl_rank, int* rccl_world);
/* test hook: the next runner step of the sharded schedule stalls `seconds` (<= 60) on the device
 * after its collectives and before it publishes its result (exercises sfx_runner_wait_timeout). */
int sfx_debug_stall(sfx_t h, double seconds);

/* ---------------------------------------------------------------------------------------
 * Heads sharded across ranks (BASELINE config C4: 64 tasks, 8 per GPU).
 * This handle's T heads are the global heads [head_offset, head_offset + T) of T_glob; w has
 * T_glob rows (replicated: load every task's w on every rank).  One all-task env step
 * (agents/sfdqn.py:47-60, exact in-order semantics) is the sequence below, with the caller
 * running all-reduce(MAX) over ranks on X, Y (sortable int32 [T_glob][B][A]) and key (int64) in between:
 *   begin; for r < R: td_maxima(r, X), AR(X), td_update(r, X); ver_maxima(R-1, Y), AR(Y);
 *   verify(X, Y, flag) -> while flag < T_glob: one more round r = R, R+1, ... (td_maxima,
 *   AR, td_update, ver_maxima, AR, verify);  select(r_last, task, use_gpi, key), AR(key);
 *   finish(rounds run).
 * key decodes as idx = 0xFFFFFFFF - ((key ^ 2^63) & 0xFFFFFFFF): c = idx / A, a = idx % A
 * (SF.GPI + argmax with first-index ties, features/successor.py:223-273).
 * ------------------------------------------------------------------------------------- */
int sfx_shard_setup(sfx_t h, int T_glob, int head_offset);
/* B = 0: no minibatch (LMS + forward of s_next only; then select with round -1) */
int sfx_shard_begin(sfx_t h, const float* S_dev, const int64_t* a_dev, const float* phi_dev,
                    const float* S1_dev, const float* gamma_dev, int B, int lms_task,
                    const float* lms_phi_dev, const float* lms_r_dev, float lms_alpha,
                    const float* s_next_dev);
int sfx_shard_td_maxima(sfx_t h, int round, int32_t* X_dev);
int sfx_shard_td_update(sfx_t h, int round, const int32_t* X_dev);
int sfx_shard_ver_maxima(sfx_t h, int round, int32_t* Y_dev);
int sfx_shard_verify(sfx_t h, const int32_t* X_dev, const int32_t* Y_dev, int* flag_dev);
int sfx_shard_select(sfx_t h, int round, int task, int use_gpi, long long* key_dev);
int sfx_shard_finish(sfx_t h, int rounds_run);

/* ---------------------------------------------------------------------------------------
 * TSF-DQN (tsfdqn.py:588-709; tsfdqn_nf.py with planar-flow g): transformed features
 *   φ̃ = (h(g_i(s)) + h(g_i(s1))) ⊙ φ,  g_i = K planar flows + Linear(n_s, G), h = Linear(G, d)
 * shared by all tasks; TD target φ̃ + γ ψ⁻_i(s1)[a'], loss = l1 + β MSE(w_i·φ̃, r), one Adam step
 * over {ψ_i, w_i, g_i, h} (h's moments per task).  g packing per task: for each flow k
 * weight[n_s], bias, scale[n_s] (tsfdqn_nf.py:335-337 registration order), then Linear
 * weight[G][n_s], bias[G].  h packing: weight[d][G], bias[d].  K = 0: tsfdqn.py's g.
 * ------------------------------------------------------------------------------------- */
int sfx_tsf_setup(sfx_t h, int G, int K, float beta, double lr_g, double wd_g, double lr_h, double wd_h);
/* Planar flows held fixed (Adam with lr = 0 on the flow parameters; the Linear of g_i and h still
 * train): mirrors tsfdqn_nf.py on a GPU, where PlanarFlow's Parameter(...).to(device) leaves the
 * flows unregistered, so the reference's optimizer never updates them. */
int sfx_tsf_freeze_flows(sfx_t h, int freeze);
int sfx_tsf_load_g(sfx_t h, int t, const float* g_host);
int sfx_tsf_get_g(sfx_t h, int t, float* g_host, float* gm_host, float* gv_host);
int sfx_tsf_load_h(sfx_t h, const float* h_host);
int sfx_tsf_get_h(sfx_t h, float* h_host);
/* Checkpoint resume (sfx.checkpoint): g_t with its Adam moments; task t's Adam moments of the
 * shared h (every task's optimizer holds its own, tsfdqn.py:255-270). */
int sfx_tsf_load_g_state(sfx_t h, int t, const float* g_host, const float* gm_host, const float* gv_host);
int sfx_tsf_get_h_state(sfx_t h, int t, float* hm_host, float* hv_host);
int sfx_tsf_load_h_state(sfx_t h, int t, const float* hm_host, const float* hv_host);
/* TSFDQN.update_successor(transitions, policy, use_gpi): losses_dev [3] = (l1 + β l2, l1, l2) */
int sfx_tsf_update(sfx_t h, int policy, const float* S_dev, const int64_t* a_dev, const float* r_dev,
                   const float* phi_dev, const float* S1_dev, const float* gamma_dev, int B, int use_gpi,
                   float* losses_dev, int64_t* next_dev);

/* TSF test tasks.  A test task mixes the source tasks with ω (omega_dev [T],
 * the reference's [1, T, 1, 1] tensor) and fits its reward weights w_dev [d] and ω by Adam.
 * sfx_tsf_test_action: TSFDQN.get_test_action's greedy branch (tsfdqn.py:859-870),
 *   a_dev [1] = argmax_a w·Σ_t ω̂_t ψ_t(s)[a], ω̂ = ω / Σω (first index on ties).
 * sfx_tsf_test_update: TSFDQN.update_test_reward_mapper (tsfdqn.py:917-997) for the transition
 *   (s, a, r, φ, s1) and the next test action a1: l1 = MSE(Σ ω̂ ψ_t(s)[a], φ̃ + γ Σ ω̂ ψ⁻_t(s1)[a1]),
 *   l2 = (w·φ̃ - r)², loss = l1 + β l2 + lasso·Σ|ω|, φ̃ = φ ⊙ (h(Σ ω̂ g_t(s)) + h(Σ ω̂ g_t(s1)));
 *   one Adam step (number `step`, 1-based) on w (lr_w, wd_w) and ω (lr_omega, wd_omega) with
 *   their moments in adam_state_dev [2d + 2T] (m_w, v_w, m_ω, v_ω; zeros initially), then
 *   ω >= 1e-7.  losses_dev [3] = (loss, l2, l1), the reference's return order.  a_dev / a1_dev
 *   are device int64 scalars (the agent's action tensors).  After sfx_tsf_setup. */
/* ---------------------------------------------------------------------------------------
 * Learned φ: features/deep_phi.py DeepSF_PHI.update_successor (:93-224), the
 * library of main_sfdqn_phi_torch.py (agents/sfdqn_phi.py).  φ = phi_net(s ⊕ a ⊕ s1), an MLP
 * Linear(2 n_s + 1, hid) + ReLU, n_mid × (Linear(hid, hid) + ReLU), Linear(hid, d) with
 * hid = width_mul (2 n_s + 1) (phi_model_lambda: width_mul 2, n_mid 3), shared by the tasks; the
 * reward model of task t is Linear(d, 1) WITH bias: weight = the handle's w row t, bias and the
 * agent's loss coefficient λ_t in caller-owned device scalars.  sfx_phi_update(i): φ of the minibatch, GPI (or own-ψ)
 * next actions, targets φ + γ ψ⁻_i(s1)[a'] (they carry φ's gradient), loss = MSE(w_i(φ), r) +
 * λ_i MSE(ψ_i(s), merged), one step of a freshly built Adam (lr, moments zero, step 1 -- as the
 * reference builds torch.optim.Adam inside every update) on ψ_i, the φ net, w_i and its bias,
 * ascent on λ_i, λ_i clamped to [1e-2, 1e6]; target sync as sfx_update.  losses_dev [4] = (loss,
 * psi_loss, phi_loss, λ_i after the step), the reference's return values.
 * Packing of the φ net: torch parameters() order (W [out][in], b [out] per Linear). */
int sfx_phi_setup(sfx_t h, int width_mul, int n_mid, float lr);
int sfx_phi_numel(sfx_t h);
int sfx_phi_load(sfx_t h, const float* params_host);
int sfx_phi_get(sfx_t h, float* params_host);
/* bias_dev / lambda_dev: device scalars of the policy's reward-model bias and loss coefficient λ
 * (caller-owned, e.g. the agent's tensors), updated in place. */
int sfx_phi_update(sfx_t h, int policy, const float* S_dev, const int64_t* a_dev, const float* r_dev,
                   const float* S1_dev, const float* gamma_dev, int B, int use_gpi, float* bias_dev, float* lambda_dev,
                   float* losses_dev, int64_t* next_dev);

int sfx_tsf_test_action(sfx_t h, const float* s_dev, const float* w_dev, const float* omega_dev, int64_t* a_dev);
int sfx_tsf_test_update(sfx_t h, const float* s_dev, const float* s1_dev, const int64_t* a_dev, const int64_t* a1_dev,
                        float r, const float* phi_dev, float* w_dev, float* omega_dev, float* adam_state_dev,
                        int step, float gamma, float beta, float lasso, float lr_w, float wd_w, float lr_omega,
                        float wd_omega, float* losses_dev);
/* Lockstep test phase (SURVEY §8f rank 3 for the TSF agents: agents/tsfdqn_sequential.py:392-433,
 * tsfdqn.py:872-915 -- the E test tasks' episodes stepped together).  Row e is test task e:
 * S_dev / S1_dev [E][n_s], W_dev rows at w_stride (>= d), Omega_dev rows at o_stride (>= T),
 * adam_state_dev rows at mom_stride (>= 2d + 2T), E <= max_batch.
 * sfx_tsf_test_actions: a_dev [E] = sfx_tsf_test_action of every row, one launch set.
 * sfx_tsf_test_updates: sfx_tsf_test_update of every row (a_dev / a1_dev [E], phi_dev [E][d],
 *   losses_dev [E][3]); rowp_dev [E][6] holds each task's r, lr_w, wd_w, lr_omega, wd_omega and
 *   its 1-based Adam step (as a float) -- each test task owns its optimizer and LR schedule
 *   (agents/tsfdqn_sequential.py:333-348). */
int sfx_tsf_test_actions(sfx_t h, const float* S_dev, int E, const float* W_dev, int w_stride, const float* Omega_dev,
                         int o_stride, int64_t* a_dev);
int sfx_tsf_test_updates(sfx_t h, int E, const float* S_dev, const float* S1_dev, const int64_t* a_dev,
                         const int64_t* a1_dev, const float* phi_dev, float* W_dev, int w_stride, float* Omega_dev,
                         int o_stride, float* adam_state_dev, int mom_stride, const float* rowp_dev, float gamma,
                         float beta, float lasso, float* losses_dev);

/* ---------------------------------------------------------------------------------------
 * TSF-DQN with the source-task heads sharded across ranks (BASELINE config C5: tsfdqn_nf.py,
 * 32 tasks over 4 GPUs).  After sfx_shard_setup and sfx_tsf_setup; `policy` and
 * `task` are global indices; w (T_glob rows) and h are replicated, g_i and h's Adam moments
 * live with the policy's owner.  One TSFDQN.update_successor(transitions, i, use_gpi)
 * (tsfdqn.py:588-709) is
 *   use_gpi: every rank sfx_shard_tsf_maxima(i, S1, own_only 0, X), all-reduce(X, MAX)
 *   else:    the owner  sfx_shard_tsf_maxima(i, S1, own_only 1, X)
 *   the owner: sfx_shard_tsf_update(i, ..., X, losses); sfx_shard_tsf_shared(i, buf, 0)
 *   broadcast(buf [Ph + d], from the owner); the others sfx_shard_tsf_shared(i, buf, 1)
 * and the env action (tsfdqn.py get_Q_values: SF.GPI with w of the active task):
 *   sfx_shard_tsf_select(s, task, use_gpi, key); all-reduce(key, MAX); key decodes as for
 *   sfx_shard_select.
 * ------------------------------------------------------------------------------------- */
/* X_dev [B][A]: max over this rank's heads (own_only: the policy's own head) of ψ_t(S1)·w_policy */
int sfx_shard_tsf_maxima(sfx_t h, int policy, const float* S1_dev, int B, int own_only, int32_t* X_dev);
int sfx_shard_tsf_update(sfx_t h, int policy, const float* S_dev, const int64_t* a_dev, const float* r_dev,
                         const float* phi_dev, const float* S1_dev, const float* gamma_dev, int B,
                         const int32_t* X_dev, float* losses_dev);
/* unpack 0: buf_dev [Ph + d] <- (h, w_policy); 1: (h, w_policy) <- buf_dev */
int sfx_shard_tsf_shared(sfx_t h, int policy, float* buf_dev, int unpack);
int sfx_shard_tsf_select(sfx_t h, const float* s_dev, int task, int use_gpi, long long* key_dev);

#ifdef __cplusplus
}
#endif
#endif /* SFX_H */
