"""Process-group setup for multi-GPU providers (one process per GPU).

``init_tp_engine`` is called in every rank of a ``torchrun`` launch:
* the default group uses the ``nccl`` backend (= RCCL on ROCm) on GPUs, gloo on CPU;
* a gloo group carries the per-step metadata broadcast from rank 0 (R4);
* the TP communicator is :class:`RcclComm` on GPUs (graph-capturable), or
  :class:`TorchComm` over gloo on CPU (tests).
Rank 0 owns the scheduler and the provider node; ranks 1..N-1 call
``engine.runner.worker_loop()``.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .comm import HostStagedComm, RcclComm, TorchComm, XgmiComm


def init_distributed(backend: str | None = None) -> tuple[int, int, int]:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        local = local % torch.cuda.device_count()  # several ranks per GPU: host-staged rehearsal
    if world > 1 and not dist.is_initialized():
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
        staged = os.environ.get("SYMMETRY_TP_COMM", "rccl").lower() == "gloo"
        backend = backend or ("nccl" if torch.cuda.is_available() and not staged else "gloo")
        kw = {"device_id": torch.device("cuda", local)} if backend == "nccl" else {}
        dist.init_process_group(backend, **kw)
    return rank, world, local


def make_comms(on_gpu: bool, device=None):
    """TP/EP communicator + the gloo metadata group.  ``SYMMETRY_TP_COMM=gloo`` on GPUs selects the
    host-staged communicator (ranks sharing one GPU for kernel checks; no hipGraphs).  On GPUs the
    decode-sized all-reduces run on the one-shot xGMI kernel (:class:`XgmiComm`) unless
    ``SYMMETRY_XGMI=0``; ``SYMMETRY_XGMI_SLOT`` sets its per-rank slot (bytes, default 4 MiB).

    Over the host-staged communicator the xGMI kernels are opt-in (``SYMMETRY_XGMI=1``): ranks sharing one
    GPU only make progress if their spinning kernels are co-resident, which separate processes do not
    guarantee (a miss costs the kernel's 2 s wait limit, then an error).  ``SYMMETRY_XGMI_GRAPHS=1``
    additionally lets such a rehearsal capture decode hipGraphs (every decode collective then runs on the
    xGMI kernels; a host-staged fallback inside a capture fails loudly)."""
    cpu_group = dist.new_group(backend="gloo")
    if not on_gpu:
        return TorchComm(cpu_group), cpu_group
    staged = os.environ.get("SYMMETRY_TP_COMM", "rccl").lower() == "gloo"
    comm = HostStagedComm(cpu_group) if staged else RcclComm(bootstrap_group=cpu_group)
    want = os.environ.get("SYMMETRY_XGMI", "auto")
    if (want == "1" or (want == "auto" and not staged)) and 1 < comm.world <= 8:
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        xg = _try_xgmi(comm, cpu_group, dev)
        if xg is not None:
            comm = xg
            if staged and os.environ.get("SYMMETRY_XGMI_GRAPHS", "0") == "1":
                comm.capturable = True
    return comm, cpu_group


def _try_xgmi(inner, group, dev):
    """The xGMI communicator on every rank, or on none: a rank whose peer-memory mapping fails (IPC refused,
    no peer access) votes no over the gloo group and every rank keeps the plain RCCL communicator."""
    import sys

    xg, err = None, None
    try:
        xg = XgmiComm(inner, group, dev, int(os.environ.get("SYMMETRY_XGMI_SLOT", 4 << 20)), barrier=False)
    except Exception as exc:  # noqa: BLE001 -- any failure means: no one-shot kernels on this node
        err = exc
    if _vote(xg is not None, group):
        dist.barrier(group=group)  # every rank mapped every buffer before the first collective
        # a startup all-reduce of known values: links / mappings that misbehave cost one wait limit here and a
        # fallback to RCCL, not the first decode step
        passed = False
        try:
            passed = xg.self_test()
        except Exception as exc:  # noqa: BLE001
            err = exc
        if _vote(passed, group):
            return xg
        err = err or RuntimeError("startup all-reduce self-test failed")
    if err is not None:
        print(f"symmetry: xGMI one-shot collectives unavailable ({type(err).__name__}: {err}); using RCCL",
              file=sys.stderr, flush=True)
    if xg is not None:
        xg.destroy(inner_too=False)
    return None


def _vote(ok: bool, group) -> bool:
    """True on every rank iff ``ok`` on every rank (gloo)."""
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return int(t[0]) == 1


def _attach_xar_checked(comm, group, d: int, ks=(256,)) -> None:
    """attach_xar + its startup self-test on every rank; on any failure every rank drops the fused path (the
    decode step then runs GEMM + the one-shot all-reduce)."""
    import sys

    attached, passed, err = False, False, None
    try:
        comm.attach_xar(group, 64, d)
        attached = True
    except Exception as exc:  # noqa: BLE001
        err = exc
    if _vote(attached, group):
        dist.barrier(group=group)  # every rank mapped every peer slot before the first fused launch
        try:
            # the production shapes: the row-parallel K of o and down, 1 and 16 rows, both weight layouts
            passed = comm.xar_self_test(d, ks=ks, rows=(1, 16), layouts=(False, True))
        except Exception as exc:  # noqa: BLE001
            err = exc
        if _vote(passed, group):
            return
    print(f"symmetry: fused GEMM + all-reduce launches disabled ({err or 'startup self-test failed'})",
          file=sys.stderr, flush=True)
    if comm.xar is not None:
        comm.xar.destroy(inner_too=False)
        comm.xar = None


def a2a_capacity(tokens: int, world: int) -> int:
    """Rows one rank may push to one token-slice owner in the replicated-token expert exchange: one pre-combined
    row per token of the owner's slice, ceil(T / N) (models/moe.py forward_a2a)."""
    return -(-int(tokens) // world)


def _attach_a2a_checked(comm, group, tokens: int, mcfg, world: int) -> None:
    """attach_a2a on every rank or on none: a rank whose uncached allocation or IPC mapping fails votes no over
    gloo, every rank drops the communicator, and MoE prefill combines by all-reduce instead."""
    import sys

    ok, err = False, None
    try:
        comm.attach_a2a(group, a2a_capacity(tokens, world), mcfg.hidden_size * 4)
        ok = True
    except Exception as exc:  # noqa: BLE001
        err = exc
    if _vote(ok, group):
        dist.barrier(group=group)  # every rank mapped every peer slot before the first exchange
        return
    print(f"symmetry: xGMI expert all-to-all unavailable ({err or 'a peer failed to attach'}); "
          "MoE prefill combines by all-reduce", file=sys.stderr, flush=True)
    if comm.a2a is not None:
        comm.a2a.destroy(inner_too=False)
        comm.a2a = None


def init_tp_engine(ecfg):
    """Build this rank's engine shard; returns (engine, rank).

    Dense models: tensor parallel over all ranks.  MoE models (Mixtral, BASELINE config 5): attention
    tensor parallel over all ranks and the experts expert-parallel over the same ranks (E / world experts
    per GPU), sharing one communicator; the expert outputs are combined by all-reduce (tokens are
    replicated by the TP attention) or all-to-all dispatch (``moe.mode = "a2a"``).
    """
    from ..engine.llm_engine import LLMEngine
    from ..models.config import resolve

    rank, world, local = init_distributed()
    on_gpu = torch.cuda.is_available() and ecfg.device != "cpu"
    comm, cpu_group = make_comms(on_gpu, torch.device("cuda", local) if on_gpu else None)
    ecfg.tp_size, ecfg.tp_rank = world, rank
    mcfg = ecfg.model_config or resolve(ecfg.model)
    ep_comm = None
    if mcfg.is_moe and world > 1:
        if mcfg.num_experts % world:
            raise ValueError(f"{mcfg.num_experts} experts do not shard over {world} ranks")
        ecfg.ep_size, ecfg.ep_rank = world, rank
        ep_comm = comm
    if on_gpu:
        ecfg.device = f"cuda:{local}"
    xar = os.environ.get("SYMMETRY_XGMI_FUSED", "1")
    if isinstance(comm, XgmiComm) and xar != "0" and (torch.cuda.device_count() >= world or xar == "force"):
        # the fused row-parallel decode projections (GEMM + all-reduce + residual in one launch): <= 64 rows.  Not
        # when ranks share a GPU (the one-GPU rehearsal): a fused launch's workgroups wait for the other ranks'
        # tiles while holding their CUs, and one rank's grid can fill the whole device before the other's starts
        # (SYMMETRY_XGMI_FUSED=force: a test whose grids are small enough to be co-resident anyway)
        ks = {mcfg.num_heads * mcfg.head_dim // world}
        if not mcfg.is_moe:
            ks.add(mcfg.intermediate_size // world)
        _attach_xar_checked(comm, cpu_group, mcfg.hidden_size, ks=tuple(sorted(k for k in ks if k % 256 == 0)) or (256,))
    a2a = os.environ.get("SYMMETRY_MOE_XGMI_A2A", "1")
    if ep_comm is not None and isinstance(comm, XgmiComm) and a2a != "0" and (
            torch.cuda.device_count() >= world or a2a == "force"):
        # the unpadded expert all-to-all (prefill: expert results pushed to the token-slice owners) on its own
        # peer buffers, sized by the largest prefill step.  Not when ranks share a GPU (the one-GPU rehearsal,
        # bench/ep_rehearsal.py): a rank's spinning exchange grid holds CUs its peers need to arrive -- at 4 ranks
        # a 256-token Mixtral step hit the wait limit (profiles/r6/ep_crossover.jsonl); the counted RCCL / gloo
        # exchange runs instead (SYMMETRY_MOE_XGMI_A2A=force: tests whose grids are small enough)
        _attach_a2a_checked(comm, cpu_group, ecfg.max_num_batched_tokens, mcfg, world)
    engine = LLMEngine(ecfg, tp_comm=comm, ep_comm=ep_comm, cpu_group=cpu_group)
    if rank == 0 and world > 1:
        # fault containment: a lost worker takes the provider offline within ~0.1 s (parallel/health.py)
        from .health import TPHealthMonitor

        engine.health = TPHealthMonitor(engine.runner.meta, comm,
                                        period_s=float(os.environ.get("SYMMETRY_HEALTH_PERIOD_S", "0.1")))
        engine.health.add_listener(engine.declare_fatal)
        engine.health.start()
    return engine, rank
