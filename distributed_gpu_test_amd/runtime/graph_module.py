"""The engine's module forward and backward replayed from HIP graphs under the eager API.

DeepSpeed users drive a step as ``loss = crit(engine(x), y); engine.backward(loss); engine.step()``
(reference ``train.py:110-114``).  Eagerly, every op of the module is one host launch and one
autograd node, so a small model is host-bound (~300-400 us per step for the reference MLP).  With
``"amd": {"graph_module": true}`` the engine captures, per input signature:

* a forward graph: ``static_out = module(*static_in)``;
* a backward graph: ``autograd.grad(static_out, params, static_gout)`` followed by an in-graph
  ``grad_view.add_(g)`` into the engine's flat gradient buckets — the accumulation autograd's
  ``AccumulateGrad`` would otherwise launch once per parameter.

``engine(x)`` then copies ``x`` into the static input and replays the forward graph; the user's
loss runs eagerly; ``engine.backward`` reaches ``_Replay.backward``, which copies the incoming
gradient and replays the backward graph.  ``_Replay`` returns no gradient for the parameters, so
autograd runs their ``AccumulateGrad`` nodes with an undefined gradient: nothing is added twice and
the post-accumulate hooks (the bucket reducer: all-reduce / reduce-scatter overlapped with the rest
of backward) still fire, as for the fused Linear kernels (``ops/linear.py``).

Same kernels, same accumulation order: the trajectory matches the eager engine.  The warmup runs
before capture execute the module for real, so the module's buffers (BatchNorm running stats,
``num_batches_tracked``) and the CPU / GPU RNG states are saved before them and restored after.
The returned outputs alias the static output buffers (overwritten by the next replay of that
signature), as with ``torch.cuda.make_graphed_callables``; so a signature's graph is only
replayed once its previous forward's backward has run (``pending``): a second forward of the same
signature before that runs eagerly instead of overwriting the first one's activations.
"""
from __future__ import annotations

import gc
from typing import Callable, List, Optional, Sequence, Tuple

import torch


def _as_tuple(out) -> Tuple[torch.Tensor, ...]:
    if torch.is_tensor(out):
        return (out,)
    if isinstance(out, (tuple, list)) and all(torch.is_tensor(o) for o in out):
        return tuple(out)
    raise TypeError(f"graph_module needs a module returning a tensor or a tuple of tensors, got {type(out).__name__}")


_CAPTURE_STREAMS: dict = {}

# A graph replay costs ~10 us of device time on this stack whatever it holds, and in most processes
# the host blocks on it; one kernel launched directly costs ~4-5 us (profiles/r5_graph_launch_cost.txt).
# A graph that captured at most this many kernels (in a chain, nothing else: no copy, memset, event
# or collective) is therefore run as those kernels re-launched with the captured arguments, in one
# C++ call (``_C.DirectLaunch``): the forward, the graphed tail and the whole-step graph of a small
# model (profiles/r5_graph_direct_ab.txt: graph_module 17-22k -> 26-30k iters/s, whole-step graph
# 34-35k -> 38-46k on the reference model).  DGT_GRAPH_DIRECT=0 keeps every replay, and a graph
# that consumes RNG is always replayed (``rng_checked``).
DIRECT_MAX_KERNELS = 8


def direct_launcher(graph: "torch.cuda.CUDAGraph", may_hold_collective: bool = True):
    """``_C.DirectLaunch`` for a ``keep_graph=True`` graph of at most DIRECT_MAX_KERNELS chained
    kernels (DGT_GRAPH_DIRECT_MAX overrides the limit), else None (then replay it).  The graph object
    must outlive the launcher: it owns the captured kernel arguments.  ``may_hold_collective``: the
    graph was captured where a collective can run (the graphed tail, the whole-step graph); with
    more than one rank such a graph is only replayed."""
    import os
    if os.environ.get("DGT_GRAPH_DIRECT", "1") == "0":
        return None
    limit = int(os.environ.get("DGT_GRAPH_DIRECT_MAX", DIRECT_MAX_KERNELS))
    if may_hold_collective and torch.distributed.is_available() and torch.distributed.is_initialized() \
            and torch.distributed.get_world_size() > 1:
        return None  # a captured collective's kernels are only ever replayed (its plan lives in RCCL)
    from ..ops import _ext
    try:
        mod = _ext.fast()
    except Exception:  # no extension: replay
        return None
    if not hasattr(mod, "graph_direct_plan"):
        return None
    raw = getattr(graph, "raw_cuda_graph", None)
    if raw is None:  # (a torch without it: replay; compat.py reports the missing feature)
        return None
    plan = mod.graph_direct_plan(int(raw()), torch.cuda.current_device())
    if plan is None or plan.kernels > limit:
        return None
    return plan


def rng_checked(graph: "torch.cuda.CUDAGraph", direct, install: Callable[[Callable[[], None]], None]):
    """The callable that runs ``graph``: its first call is a real ``replay()``, which also refills the
    graph's captured Philox seed / offset and advances the CUDA generator (dropout, ``torch.rand``
    inside the graph).  A direct launcher (``direct_launcher``) re-launches the captured kernels
    with their captured arguments and does neither, so it would hand a graph that draws random
    numbers the same numbers on every step.  Only a graph whose first replay left the default
    generator's state unchanged -- it consumes no RNG -- switches to ``direct``: ``install`` receives
    the callable every later call should use (the direct launcher or the bound replay)."""
    replay = torch._C._CUDAGraph.replay.__get__(graph)
    if direct is None:
        return replay

    def first() -> None:
        before = torch.cuda.get_rng_state()
        replay()
        install(direct if torch.equal(before, torch.cuda.get_rng_state()) else replay)
    return first


def _setter(obj, attr: str):
    """``install`` for rng_checked that holds ``obj`` weakly: a strong reference from the callable
    stored on ``obj`` back to ``obj`` would be a cycle, and a cycle holding HIP graphs is freed by the
    garbage collector whenever it runs -- possibly inside another graph's capture, where destroying a
    graph aborts the process.  Without the cycle the graphs go when their owner does."""
    import weakref
    ref = weakref.ref(obj)

    def install(f) -> None:
        o = ref()
        if o is not None:
            setattr(o, attr, f)
    return install


class _capture:
    """``torch.cuda.graph`` without its ``gc.collect()`` + ``empty_cache()`` on entry: emptying the
    caching allocator moves every later allocation, so the addresses bound graphs were captured for
    (``bind_inputs``) would never come back.  Captures on one side stream per device, ordered
    after and before the caller's stream."""

    __slots__ = ("graph", "pool", "stream", "ctx", "gc_was_on")

    def __init__(self, graph: "torch.cuda.CUDAGraph", pool):
        self.graph, self.pool = graph, pool
        dev = torch.cuda.current_device()
        self.stream = _CAPTURE_STREAMS.get(dev)
        if self.stream is None:
            self.stream = _CAPTURE_STREAMS[dev] = torch.cuda.Stream()

    def __enter__(self):
        self.stream.wait_stream(torch.cuda.current_stream())
        self.ctx = torch.cuda.stream(self.stream)
        self.ctx.__enter__()
        # no garbage collection while capturing: a collected cycle that owns HIP graphs, events or
        # streams (any user object) would destroy them mid-capture, which aborts the process
        self.gc_was_on = gc.isenabled()
        gc.disable()
        try:
            self.graph.capture_begin(pool=self.pool)
        except BaseException:
            if self.gc_was_on:
                gc.enable()
            raise
        return self

    def __exit__(self, *exc):
        try:
            self.graph.capture_end()
        finally:
            if self.gc_was_on:
                gc.enable()
            self.ctx.__exit__(*exc)
            torch.cuda.current_stream().wait_stream(self.stream)
        return False


class GraphedModule:
    def __init__(self, module: torch.nn.Module, params: Sequence[torch.nn.Parameter], args: Sequence[torch.Tensor],
                 warmup: int = 2, tail: Optional[Callable[[], None]] = None, bind_inputs: bool = False):
        self.params: List[torch.nn.Parameter] = list(params)
        self.grad_views = [p.grad for p in self.params]
        if any(g is None or g.shape != p.shape for g, p in zip(self.grad_views, self.params)):
            raise RuntimeError("graph_module needs the engine's gradient views bound (.grad) before capture")
        # bind_inputs: the graphs read the caller's input tensors where they lie (no static copy);
        # replayed only for inputs at the same addresses (``bound_ptrs``), see Engine._graphed_forward
        self.bound_ptrs = None
        if bind_inputs:
            if any(a.requires_grad or not a.is_contiguous() for a in args):
                raise ValueError("bind_inputs needs contiguous inputs that do not require grad")
            self.static_in = tuple(a.detach() for a in args)
        else:
            self.static_in = tuple(a.detach().clone().requires_grad_(a.requires_grad) for a in args)
        self.in_rg = [i for i, a in enumerate(self.static_in) if a.requires_grad]
        # The graphs run the module on ALIASES of its parameters (same storage, so optimizer updates
        # are seen, but separate autograd leaves): capture never touches the real parameters'
        # AccumulateGrad nodes.  Those are created by the eager _Replay on the caller's stream;
        # created on a capture stream they would put a cross-stream wait into every later backward
        # (and, during capture, an event wait on a non-capturing stream).
        by_id = {id(p): n for n, p in module.named_parameters()}
        self._param_ix = {id(p): i for i, p in enumerate(self.params)}
        if any(id(p) not in by_id for p in self.params):
            raise RuntimeError("graph_module: every trained tensor must be a parameter of the module")
        self.aliases = {n: p.detach().requires_grad_(p.requires_grad) for n, p in module.named_parameters()}
        targets = [self.aliases[by_id[id(p)]] for p in self.params] + [self.static_in[i] for i in self.in_rg]

        def run():
            return _as_tuple(torch.func.functional_call(module, self.aliases, self.static_in))

        if warmup:
            cur = torch.cuda.current_stream()
            side = torch.cuda.Stream()
            side.wait_stream(cur)
            # the warmup executes the module: keep its buffers and the RNG streams as they were
            bufs = [(b, b.detach().clone()) for b in module.buffers()]
            cpu_rng, gpu_rng = torch.get_rng_state(), torch.cuda.get_rng_state()
            with torch.cuda.stream(side):  # library handles / workspaces before capture
                for _ in range(warmup):
                    outs = [o for o in run() if o.requires_grad]
                    torch.autograd.grad(outs, targets, grad_outputs=[torch.ones_like(o) for o in outs],
                                        allow_unused=True)
                    del outs
            cur.wait_stream(side)
            with torch.no_grad():
                for b, saved in bufs:
                    b.copy_(saved)
            torch.set_rng_state(cpu_rng)
            torch.cuda.set_rng_state(gpu_rng)
        self.pool = torch.cuda.graph_pool_handle()
        self.fwd = torch.cuda.CUDAGraph(keep_graph=True)  # (kept: a direct launcher reads its kernel nodes)
        with _capture(self.fwd, self.pool):
            out = run()
            self.grad_out_idx = [i for i, o in enumerate(out) if o.requires_grad]
            # allocated in the graph's pool, not the caller's: a block taken from the caching
            # allocator here would shift the addresses the caller's next batches land at
            self.static_gout = [torch.empty_like(out[i]) for i in self.grad_out_idx]
        self.static_out = out
        self.fwd.instantiate()
        self.fwd_direct = direct_launcher(self.fwd, may_hold_collective=False)
        self.bwd = torch.cuda.CUDAGraph(keep_graph=True)
        # The injected HIP Linear kernels (ops/linear.py, ops/mfma_linear.py) add dW / db straight into
        # their parameter's .grad inside an engine backward: with the aliases' .grad bound to the
        # engine's gradient views, the captured backward needs no separate add per parameter (one
        # graph node each); parameters of other modules still come back from autograd and are added.
        from ..ops.linear import engine_backward
        for n, p in module.named_parameters():
            if id(p) in self._param_ix:
                self.aliases[n].grad = self.grad_views[self._param_ix[id(p)]]
        # a tail (below) captures this backward a second time, so keep the autograd graph for it
        with_tail = tail is not None and not self.in_rg
        with _capture(self.bwd, self.pool), engine_backward(False):
            gs = torch.autograd.grad([out[i] for i in self.grad_out_idx], targets, grad_outputs=self.static_gout,
                                     allow_unused=True, retain_graph=with_tail)
            with torch.no_grad():
                for gv, g in zip(self.grad_views, gs[:len(self.params)]):
                    if g is not None:
                        gv.add_(g)
        self.static_gin = gs[len(self.params):]
        self.bwd.instantiate()
        self.bwd_direct = direct_launcher(self.bwd, may_hold_collective=False)  # (the reducer runs outside)
        self.bwd_replay = rng_checked(self.bwd, self.bwd_direct, _setter(self, "bwd_replay"))
        # The graphed tail: the same backward followed by ``tail()`` (the engine's gradient
        # collective, clip coefficient, fused Adam, ZeRO-1 all-gather and the bucket's zero fill) in
        # ONE graph, replayed by Engine.backward when the loss is one it can differentiate itself
        # (the framework's fused BCE on this module's output): a training step is then the forward
        # replay, the loss kernel and this replay, with no autograd engine call at all.
        self.bwd_tail = None
        self.tail_lr = getattr(tail, "lr", None)  # baked into the captured Adam launch
        if with_tail:
            self.bwd_tail = torch.cuda.CUDAGraph(keep_graph=True)
            with _capture(self.bwd_tail, self.pool), engine_backward(False):
                gs2 = torch.autograd.grad([out[i] for i in self.grad_out_idx], targets[:len(self.params)],
                                          grad_outputs=self.static_gout, allow_unused=True)
                with torch.no_grad():
                    for gv, g in zip(self.grad_views, gs2):
                        if g is not None:
                            gv.add_(g)
                    tail()
            del gs2
        self.single = torch.is_tensor(out) or len(out) == 1
        # (bound C methods: no Python wrapper frame per step)
        # (a graph that draws random numbers is always replayed: rng_checked)
        self.fwd_replay = rng_checked(self.fwd, self.fwd_direct, _setter(self, "fwd_replay"))
        self.tail_replay = None
        if self.bwd_tail is not None:
            self.bwd_tail.instantiate()
            self.tail_direct = direct_launcher(self.bwd_tail)
            self.tail_replay = rng_checked(self.bwd_tail, self.tail_direct, _setter(self, "tail_replay"))
        self.replays = 0
        self.pending = False  # a replayed forward whose backward has not run yet
        self.held = None  # bound inputs of the pending forward: alive (and unmoved) until its backward
        if bind_inputs:
            # keep no reference to the caller's tensors: their blocks go back to the caching
            # allocator, which hands the same addresses to the next step's batch
            self.bound_ptrs = tuple(a.data_ptr() for a in self.static_in)
            self.static_in = None
        # the framework's fused BCE on this graph's (single, differentiable) output writes its
        # d loss / d logits straight into the backward graph's static input (ops/loss.py
        # claim_gout): no copy before the backward replay.  One claim per forward replay.
        self.gout_claimable = False
        if self.single and self.grad_out_idx == [0]:
            from ..ops.loss import register_gout_alias
            register_gout_alias(self.static_out[0], self)

    def claim_gout(self, z: torch.Tensor, dtype: torch.dtype) -> Optional[torch.Tensor]:
        """The static gradient input as the destination of d loss / d logits of ``z`` (this graph's
        output of the latest replay, read by its first loss), else None."""
        g = self.static_gout[0]
        if (not self.gout_claimable or not self.pending or g.dtype != dtype or z.numel() != g.numel()
                or z.data_ptr() != self.static_out[0].data_ptr()):
            return None
        self.gout_claimable = False
        return g

    def __call__(self, *args):
        grad = torch.is_grad_enabled()  # the caller's mode: inside Function.forward it is always off
        outs = _replay_apply(self, *args, *self.params)  # (a single output comes back as a tensor)
        self.pending = grad  # under no_grad no backward will come
        if self.bound_ptrs is not None:
            self.held = args if grad else None
        return outs

    def finish(self) -> None:
        """The pending forward's backward has been replayed."""
        self.pending = False
        self.held = None


class _Replay(torch.autograd.Function):
    @staticmethod
    def forward(ctx, runner: GraphedModule, *tensors):
        if runner.bound_ptrs is None:
            for dst, src in zip(runner.static_in, tensors[:len(runner.static_in)]):
                if dst.data_ptr() != src.data_ptr():
                    dst.copy_(src)
        elif (runner.bound_ptrs[0] != tensors[0].data_ptr() if len(runner.bound_ptrs) == 1
              else any(p != t.data_ptr() for p, t in zip(runner.bound_ptrs, tensors))):
            raise RuntimeError("graph_module: a bound graph replayed for inputs at other addresses")
        runner.fwd_replay()
        runner.replays += 1
        runner.gout_claimable = True
        ctx.runner = runner
        if runner.single and runner.grad_out_idx:
            return runner.static_out[0].detach()
        outs = tuple(o.detach() for o in runner.static_out)
        for i, o in enumerate(outs):
            if i not in runner.grad_out_idx:
                ctx.mark_non_differentiable(o)
        return outs[0] if runner.single else outs

    @staticmethod
    def backward(ctx, *gouts):
        r: GraphedModule = ctx.runner
        for dst, i in zip(r.static_gout, r.grad_out_idx):
            g = gouts[i]
            if g is None:
                dst.zero_()
            elif g.data_ptr() != dst.data_ptr():  # (the fused BCE may have written it in place)
                dst.copy_(g)
        r.bwd_replay()
        r.finish()
        grads_in: List = [None] * (len(r.bound_ptrs) if r.bound_ptrs is not None else len(r.static_in))
        for i, g in zip(r.in_rg, r.static_gin):
            grads_in[i] = None if g is None else g.detach().clone()
        return (None, *grads_in, *([None] * len(r.params)))


from ..utils.fnapply import fast_apply  # noqa: E402

_replay_apply = fast_apply(_Replay)
