"""ModelRunner: scheduled batch -> device metadata -> forward -> sampled token ids.

* All per-step host metadata (token ids, positions, slots, context lengths,
  block tables, sampling params) is packed into ONE pinned int32 buffer and
  moved with ONE async H2D copy.
* Decode steps replay a hipGraph captured per (batch-size bucket, context
  bucket) (``torch.cuda.CUDAGraph`` is hipGraph on ROCm): the ~200 kernel
  launches of a Llama-3-8B step become one graph launch (MI355X_MICROARCH.md
  rows **boundary** / **graph-replay-floor**).  The context bucket bounds the
  block-table width and therefore the split-KV grid of decode attention, so
  short chats do not launch thousands of empty partition workgroups.  Padded
  rows write no cache (slot -1) and read only the reserved block 0.
* Tensor parallel: rank 0 runs the scheduler; :meth:`launch` sends the
  packed metadata to the other ranks through the step-metadata plane (R4,
  SURVEY.md §2.6; a shared-memory ring, ``parallel/metaplane.py``) and the
  workers replay the same forward via :meth:`worker_loop` without ever
  synchronising their stream, so the TP decode loop is pipelined like the
  single-GPU one: every rank enqueues step N+1 while step N runs.
"""
from __future__ import annotations

import itertools
import math
import os
import sys
import time

import numpy as np
import torch

from ..models.transformer import ForwardBatch, KVCache, TransformerLM
from ..ops import _native
from .scheduler import ScheduledBatch

DECODE_BUCKETS = (1, 2, 4, 8, 12, 16, 24, 32, 48, 64, 96, 128, 160, 192, 224, 256)
MAX_DECODE_ROWS = 256  # decode rows per step (past FUSED_DECODE_ROWS: the general path, one graph per bucket)
FUSED_DECODE_ROWS = 64
CTX_BUCKETS = (512, 2048, 8192, 32768, 131072)  # tokens (multiples of the 512-token attention partition)
CMD_STOP, CMD_CAPTURE, CMD_SYNC = -1, 2, 3  # control headers of the rank-0 -> worker metadata plane
KIND_DECODE, KIND_PREFILL, KIND_PREFILL_GRAPH = 0, 1, 4  # header[0] of a step
HEADER_LEN = 7  # kind, T, rows, max_blocks, prefill tiles, real seqs, filtered-sampling flag
# Short prefills replay a hipGraph too: T padded up to one of these token buckets, the sequence count to 1/2/4.
# A 128-token Llama-3-8B prefill is ~300 launches whose eager host enqueue (3.9 ms) held the GPU back; replayed,
# 0.19 ms (one-client TTFT 8.4 -> 7.4 ms).  SYMMETRY_PREFILL_GRAPH_TOKENS (0: off) bounds the bucket.
# Captured at start-up only (capture_all: every token bucket x one sequence x every context bucket): a bucket
# captured lazily in serving cost its first request ~14 ms of TTFT (multi-turn turn 2: 6.7 -> 21 ms,
# profiles/r4/multiturn_prefill_graph_ab.jsonl); a step whose bucket was not captured runs eagerly.
_DEBUG_PREFILL = os.environ.get("SYMMETRY_DEBUG_PREFILL") == "1"


def _ints(name: str, default: str) -> tuple:
    return tuple(int(v) for v in os.environ.get(name, default).split(",") if v.strip())


PREFILL_GRAPH_BUCKETS = _ints("SYMMETRY_PREFILL_GRAPH_BUCKETS", "16,32,64,128,192,256")
PREFILL_GRAPH_SEQS = _ints("SYMMETRY_PREFILL_GRAPH_SEQS", "1,2,4")  # padding buckets of the sequence count
PREFILL_CAPTURE_SEQS = _ints("SYMMETRY_PREFILL_CAPTURE_SEQS", "1")  # the ones captured at start-up
PREFILL_GRAPH_TOKENS = int(os.environ.get("SYMMETRY_PREFILL_GRAPH_TOKENS", "256"))
_PAD_TILE_ROW = 1 << 24  # query row of a padding attention tile: past every qlen, so its workgroups exit
_SEED_MIX = 0x9E3779B97F4A7C15


def _seq_seed(seed: int, n_out: int) -> int:
    x = (seed * 0x100000001B3 + n_out * _SEED_MIX) & 0xFFFFFFFFFFFFFFFF
    x ^= x >> 29
    return x - (1 << 64) if x >= 1 << 63 else x


class _Layout:
    """Offsets of the packed int32 metadata buffer."""

    def __init__(self, T: int, nseq: int, max_blocks: int, prefill: bool, ntiles: int = 0):
        off = 0

        def take(n):
            nonlocal off
            o = off
            off += n
            return o

        self.T, self.nseq, self.max_blocks, self.ntiles = T, nseq, max_blocks, ntiles
        self.ids = take(T)
        self.src = take(T)
        self.pos = take(T)
        self.slots = take(T)
        self.ctx = take(nseq)
        self.temps = take(nseq)
        self.topk = take(nseq)
        self.topp = take(nseq)
        if off % 2:
            take(1)
        self.seeds = take(2 * nseq)
        self.step = take(2)
        self.bt = take(nseq * max_blocks)
        self.prefill = prefill
        if prefill:
            self.cu = take(nseq + 1)
            self.tiles = take(2 * ntiles)
            if off % 2:
                take(1)
            self.last = take(2 * nseq)
        self.size = off + (off % 2)

    def views(self, buf: torch.Tensor) -> dict:
        v = {
            "input_ids": buf[self.ids:self.ids + self.T],
            "src": buf[self.src:self.src + self.T],
            "positions": buf[self.pos:self.pos + self.T],
            "slot_mapping": buf[self.slots:self.slots + self.T],
            "ctx_lens": buf[self.ctx:self.ctx + self.nseq],
            "temps": buf[self.temps:self.temps + self.nseq].view(torch.float32),
            "top_k": buf[self.topk:self.topk + self.nseq],
            "top_p": buf[self.topp:self.topp + self.nseq].view(torch.float32),
            "seeds": buf[self.seeds:self.seeds + 2 * self.nseq].view(torch.int64),
            "step": buf[self.step:self.step + 2].view(torch.int64),
            "block_tables": buf[self.bt:self.bt + self.nseq * self.max_blocks].view(self.nseq, self.max_blocks),
        }
        if self.prefill:
            v["cu_q"] = buf[self.cu:self.cu + self.nseq + 1]
            v["tiles"] = buf[self.tiles:self.tiles + 2 * self.ntiles].view(self.ntiles, 2)
            v["last_idx"] = buf[self.last:self.last + 2 * self.nseq].view(torch.int64)
        return v


class ModelRunner:
    def __init__(self, model: TransformerLM, kv: KVCache, max_num_seqs: int, max_model_len: int,
                 use_graphs: bool = True, tp_group=None, tp_rank: int = 0, tp_size: int = 1, cpu_group=None,
                 max_num_tokens: int = 8192):
        self.model = model
        self.kv = kv
        self.device = model.device
        self.block_size = kv.block_size
        self.max_blocks = math.ceil(max_model_len / kv.block_size)
        self.max_num_seqs = max_num_seqs
        self.buckets = [b for b in DECODE_BUCKETS if b < max_num_seqs] + [max_num_seqs]
        self.buckets = sorted(set(b for b in self.buckets if b <= MAX_DECODE_ROWS))
        bs = kv.block_size
        self.ctx_blocks = sorted({math.ceil(min(c, max_model_len) / bs) for c in CTX_BUCKETS} | {self.max_blocks})
        self.ctx_blocks = [b for b in self.ctx_blocks if b <= self.max_blocks]
        self.is_gpu = self.device.type != "cpu"
        self.use_graphs = use_graphs and self.is_gpu
        # pad short prefills to the graph buckets (without use_graphs -- CPU tests -- they then run eagerly)
        self.prefill_graphs = self.use_graphs
        self.prefill_graph_replays = 0
        self.graph_replays = 0  # decode steps run as a replayed hipGraph
        self.tp_size, self.tp_rank = tp_size, tp_rank
        self.cpu_group = cpu_group
        self.graphs: dict[tuple, tuple] = {}
        self._graph_pool = None
        self._pinned = {}
        self.step_counter = 0
        self._parity = 0
        # host seconds per phase of launch() (TP host-phase breakdown, bench.py "host_ms_per_step"): packing the
        # metadata, the metadata plane push (TP), the H2D copy + graph replay / eager forward enqueue, the D2H
        # copy + event; "forward": launch-to-completion as seen by wait()
        self.timing = {"fill": 0.0, "send": 0.0, "run": 0.0, "graph_launch": 0.0, "d2h": 0.0, "forward": 0.0,
                       "steps": 0}
        self.meta = None
        # (tp_size > 1 without a bootstrap group: ONE rank's shard alone, no workers -- the TP shard timing
        # simulation of bench/tp_shard.py)
        if tp_size > 1 and cpu_group is not None:
            from ..parallel.metaplane import make_metaplane

            n = max(max_num_tokens, max_num_seqs)
            nseq = max(max_num_seqs, 1)
            ints = 4 * n + 12 * nseq + 2 * (n // 64 + nseq) + nseq * self.max_blocks + 64 + HEADER_LEN
            self.meta = make_metaplane(cpu_group, tp_rank, tp_size, HEADER_LEN, 4 * (ints + ints // 4) + 4096)
        self._wslots: list = []  # worker: ring of (pinned buffer, event) for the H2D copies in flight
        self._wnext = 0
        self._stop_sent = False
        self.sync_times: list[float] = []  # worker: host times of rank 0's sync points

    # ------------------------------------------------------------------------------------------
    def _host(self, n: int, key: str) -> torch.Tensor:
        t = self._pinned.get(key)
        if t is None or t.numel() < n:
            t = torch.empty(max(n, 1024), dtype=torch.int32, pin_memory=self.is_gpu)
            self._pinned[key] = t
        return t[:n]

    def _fill_decode(self, lay: _Layout, host: np.ndarray, seqs, prev_rows: dict | None) -> None:
        """_fill for a decode step (one token per sequence), vectorised: at 128-256 concurrent sequences the
        per-sequence Python of the generic packer cost more host time than the GPU step (wide batches)."""
        BS, n, T = self.block_size, len(seqs), lay.T
        host[:] = 0
        ids = np.empty(n, dtype=np.int64)
        src = np.full(T, -1, dtype=np.int64)
        pos = np.empty(n, dtype=np.int64)
        for i, s in enumerate(seqs):
            p = s.num_computed
            pos[i] = p
            npr = len(s.prompt_ids)
            if p < npr:
                ids[i] = s.prompt_ids[p]
            elif p - npr < len(s.output_ids):
                ids[i] = s.output_ids[p - npr]
            else:  # pending token (pipelined decode): resolved on the device
                ids[i] = 0
                src[i] = prev_rows[s.seq_id]
        # block tables: one flat conversion, scattered into the [rows, max_blocks] view
        lens = np.fromiter((len(s.block_table) for s in seqs), dtype=np.int64, count=n)
        flat = np.fromiter(itertools.chain.from_iterable(s.block_table for s in seqs), dtype=np.int64,
                           count=int(lens.sum()))
        btv = host[lay.bt:lay.bt + lay.nseq * lay.max_blocks].reshape(lay.nseq, lay.max_blocks)
        rows = np.repeat(np.arange(n), lens)
        cols = np.arange(flat.size) - np.repeat(np.cumsum(lens) - lens, lens)
        btv[rows, cols] = flat
        blk = btv[np.arange(n), pos // BS].astype(np.int64)
        host[lay.ids:lay.ids + n] = ids
        host[lay.src:lay.src + T] = src
        host[lay.pos:lay.pos + n] = pos
        host[lay.slots:lay.slots + n] = blk * BS + pos % BS
        host[lay.slots + n:lay.slots + T] = -1
        host[lay.ctx:lay.ctx + n] = pos + 1
        host[lay.ctx + n:lay.ctx + lay.nseq] = 1
        prm = [s.params for s in seqs]
        host[lay.temps:lay.temps + n] = np.fromiter((q.temperature for q in prm), np.float32, n).view(np.int32)
        host[lay.topk:lay.topk + n] = np.fromiter((q.top_k for q in prm), np.int64, n)
        host[lay.topp:lay.topp + lay.nseq] = np.ones(lay.nseq, dtype=np.float32).view(np.int32)
        host[lay.topp:lay.topp + n] = np.fromiter((q.top_p for q in prm), np.float32, n).view(np.int32)
        # _seq_seed, vectorised (uint64 arithmetic wraps mod 2^64 like the Python masks)
        seed = np.fromiter((s.sampling_seed & 0xFFFFFFFFFFFFFFFF for s in seqs), np.uint64, n)
        nout = np.fromiter((len(s.output_ids) for s in seqs), np.uint64, n)
        with np.errstate(over="ignore"):
            x = seed * np.uint64(0x100000001B3) + nout * np.uint64(_SEED_MIX)
        x ^= x >> np.uint64(29)
        host[lay.seeds:lay.seeds + 2 * n] = x.view(np.int32)

    def _fill(self, lay: _Layout, host: np.ndarray, seqs, counts, prev_rows: dict | None = None) -> None:
        """Pack one step's metadata.  A decode row whose input token is still in flight (sampled by the
        previous, not yet completed step: pipelined decode) gets id 0 and src = that step's output row;
        the embedding kernel then reads the token from device memory."""
        if not lay.prefill and seqs:
            self._fill_decode(lay, host, seqs, prev_rows)
        else:
            self._fill_generic(lay, host, seqs, counts, prev_rows)

    def _fill_generic(self, lay: _Layout, host: np.ndarray, seqs, counts, prev_rows: dict | None = None) -> None:
        BS = self.block_size
        ids, pos, slots, src = [], [], [], []
        ctx, temps, seeds, topk, topp = [], [], [], [], []
        for seq, n in zip(seqs, counts):
            start = seq.num_computed
            toks = seq.token_slice(start, n)
            if len(toks) < n:  # pending token (pipelined decode): resolved on the device
                toks = toks + [0] * (n - len(toks))
                src.extend([-1] * (n - 1) + [prev_rows[seq.seq_id]])
            else:
                src.extend([-1] * n)
            p = np.arange(start, start + n, dtype=np.int64)
            bt = np.asarray(seq.block_table, dtype=np.int64)
            ids.extend(toks)
            pos.append(p)
            slots.append(bt[p // BS] * BS + p % BS)
            ctx.append(start + n)
            temps.append(seq.params.temperature)
            topk.append(seq.params.top_k)
            topp.append(seq.params.top_p)
            seeds.append(_seq_seed(seq.sampling_seed, len(seq.output_ids)))
        nreal = len(seqs)
        T = lay.T
        host[:] = 0
        host[lay.ids:lay.ids + len(ids)] = ids
        host[lay.src:lay.src + T] = -1
        host[lay.src:lay.src + len(src)] = src
        if pos:
            host[lay.pos:lay.pos + len(ids)] = np.concatenate(pos)
            host[lay.slots:lay.slots + len(ids)] = np.concatenate(slots)
        host[lay.slots + len(ids):lay.slots + T] = -1
        host[lay.ctx:lay.ctx + nreal] = ctx
        host[lay.ctx + nreal:lay.ctx + lay.nseq] = 1
        host[lay.temps:lay.temps + nreal] = np.asarray(temps, dtype=np.float32).view(np.int32)
        host[lay.topk:lay.topk + nreal] = topk
        host[lay.topp:lay.topp + lay.nseq] = np.ones(lay.nseq, dtype=np.float32).view(np.int32)
        host[lay.topp:lay.topp + nreal] = np.asarray(topp, dtype=np.float32).view(np.int32)
        host[lay.seeds:lay.seeds + 2 * nreal] = np.asarray(seeds, dtype=np.int64).view(np.int32)
        btv = host[lay.bt:lay.bt + lay.nseq * lay.max_blocks].reshape(lay.nseq, lay.max_blocks)
        for i, seq in enumerate(seqs):
            btv[i, :len(seq.block_table)] = seq.block_table
        if lay.prefill:
            # padding sequences of a graph bucket: qlen 0 (cu_q repeats the real total), context 1, last row 0
            cu = np.full(lay.nseq + 1, len(ids), dtype=np.int64)
            cu[0] = 0
            cu[1:nreal + 1] = np.cumsum(counts, dtype=np.int64)
            host[lay.cu:lay.cu + lay.nseq + 1] = cu
            tiles = []
            for i, n in enumerate(counts):
                tiles.extend((i, r) for r in range(0, n, 64))
            # heaviest first (keys visible to the tile's last row): the causal tail of a long prompt starts
            # in the first wave of attention workgroups instead of finishing last
            if len(tiles) > 1:
                tiles.sort(key=lambda t: -(ctx[t[0]] - counts[t[0]] + min(t[1] + 64, counts[t[0]])))
            if tiles:
                host[lay.tiles:lay.tiles + 2 * len(tiles)] = np.asarray(tiles, dtype=np.int32).reshape(-1)
            if lay.ntiles > len(tiles):  # padding tiles (graph buckets): row past every qlen -> workgroup exits
                host[lay.tiles + 2 * len(tiles) + 1:lay.tiles + 2 * lay.ntiles:2] = _PAD_TILE_ROW
            host[lay.last:lay.last + 2 * lay.nseq] = np.maximum(cu[1:] - 1, 0).astype(np.int64).view(np.int32)

    def _forward_batch(self, kind: str, lay: _Layout, dev: torch.Tensor, nseq: int, need_logits=False,
                       filtered=False):
        v = lay.views(dev)
        return ForwardBatch(kind=kind, num_seqs=nseq, need_logits=need_logits, filtered=filtered, **v)

    @staticmethod
    def _filtered(seqs) -> bool:
        """Does any row need the full-vocab top-k / top-p sampler (temperature > 0 and a filter)?"""
        return any(s.params.temperature > 0 and (s.params.top_k > 0 or s.params.top_p < 1.0) for s in seqs)

    # ------------------------------------------------------------------------------------------
    def execute(self, batch: ScheduledBatch) -> list[int]:
        """Rank-0 entry: run one scheduled step, return sampled ids (one per sequence)."""
        return self.wait(self.launch(batch))

    def launch(self, batch: ScheduledBatch, prev_rows: dict | None = None) -> dict:
        """Enqueue one step on the GPU without waiting for it; ``wait(handle)`` returns its sampled ids.
        ``prev_rows`` maps seq_id -> output row of the in-flight previous step, for rows whose input
        token is that step's (not yet host-visible) sample."""
        seqs, counts = batch.seqs, batch.num_new_tokens
        t0 = time.perf_counter()
        filt = int(self._filtered(seqs))
        nseq = len(seqs)
        if batch.kind == "decode":
            bucket = self._bucket(nseq)
            need = max(len(s.block_table) for s in seqs)
            lay = _Layout(bucket, bucket, self._ctx_bucket(need), prefill=False)
            kind = KIND_DECODE
        else:
            T = sum(counts)
            max_blocks = max(len(s.block_table) for s in seqs)
            shape = self._prefill_graph_shape(T, nseq, max_blocks, filt)
            if shape is not None:
                lay, kind = _Layout(*shape, prefill=True, ntiles=self._pad_tiles(shape[0], shape[1])), \
                    KIND_PREFILL_GRAPH
            else:
                ntiles = sum((n + 63) // 64 for n in counts)
                lay, kind = _Layout(T, nseq, max_blocks, prefill=True, ntiles=ntiles), KIND_PREFILL
        self._parity ^= 1
        host_t = self._host(lay.size, f"{batch.kind}{self._parity}")  # double-buffered: the previous
        host = host_t.numpy()                                          # step's H2D may still be queued
        self._fill(lay, host, seqs, counts, prev_rows)
        if _DEBUG_PREFILL and batch.kind != "decode":  # the shape a prefill step's kernels see (bench diagnosis)
            bts = [b for s in seqs for b in s.block_table]
            print(f"symmetry: prefill step T={sum(counts)} seqs={nseq} new={list(counts)} "
                  f"computed={[s.num_computed for s in seqs]} blocks={[len(s.block_table) for s in seqs]} "
                  f"block ids {min(bts)}..{max(bts)} kind={kind}", file=sys.stderr, flush=True)
        header = np.array([kind, lay.T, lay.nseq, lay.max_blocks, lay.ntiles, nseq, filt], dtype=np.int32)
        t1 = time.perf_counter()
        if self.meta is not None:
            self._broadcast(header, host_t)
        t2 = time.perf_counter()
        ids = self._run(header, host_t)
        t3 = time.perf_counter()
        handle = {"nseq": nseq, "t0": t0}
        if self.is_gpu:
            pin = self._host(max(ids.numel(), 1), f"ids_out{self._parity}")[:ids.numel()]
            if _native.available() and ids.is_contiguous():
                _native.ops().copy_async(pin, ids, ids.numel() * 4, self.device.index or 0)
            else:
                pin.copy_(ids, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            handle.update(pin=pin, event=ev)
        else:
            handle["ids"] = ids.tolist()
        tm = self.timing
        tm["fill"] += t1 - t0
        tm["send"] += t2 - t1
        tm["run"] += t3 - t2
        tm["d2h"] += time.perf_counter() - t3
        tm["steps"] += 1
        return handle

    def wait(self, handle: dict) -> list[int]:
        if "event" in handle:
            handle["event"].synchronize()
            ids = handle["pin"].tolist()
            check = getattr(self.model.tp, "error", None)  # xGMI collectives: host-mapped word, no sync
            if check is not None and check():
                from ..parallel.health import TPFaultError

                raise TPFaultError("xGMI collective: a tensor-parallel peer never signalled (or was declared lost); "
                                   "this step's outputs are invalid")
        else:
            ids = handle["ids"]
        self.timing["forward"] += time.perf_counter() - handle["t0"]
        return ids[:handle["nseq"]]

    @staticmethod
    def _pad_tiles(T: int, nseq: int) -> int:
        """Attention tiles of a prefill bucket: sum(ceil(n_i / 64)) <= (T + 63 * nseq) / 64 for any split."""
        return (T + 63 * nseq) // 64

    def _prefill_graph_shape(self, T: int, nseq: int, nblocks: int, filt: int):
        """(T bucket, sequence bucket, block-table bucket) of a prefill that replays a hipGraph, or None (eager).
        One GPU, dense models: a TP prefill's collectives and the MoE dispatch stay eager."""
        if not self._prefill_graphs_on():
            return None
        Tb = next((b for b in PREFILL_GRAPH_BUCKETS if T <= b <= PREFILL_GRAPH_TOKENS), None)
        nb = next((b for b in PREFILL_GRAPH_SEQS if nseq <= b), None)
        if Tb is None or nb is None or nblocks > self.max_blocks:
            return None
        mb = self._ctx_bucket(nblocks)
        key = ("prefill", Tb, nb, mb, self._pad_tiles(Tb, nb), bool(filt))
        if self.use_graphs and key not in self.graphs:  # replay only what start-up captured
            return None
        return Tb, nb, mb

    def _prefill_graphs_on(self) -> bool:
        return self.prefill_graphs and PREFILL_GRAPH_TOKENS > 0 and self.tp_size == 1 and not self.model.cfg.is_moe

    def _bucket(self, n: int) -> int:
        for b in self.buckets:
            if b >= n:
                return b
        raise ValueError(f"decode batch {n} exceeds max_num_seqs {self.max_num_seqs}")

    def _ctx_bucket(self, nblocks: int) -> int:
        for b in self.ctx_blocks:
            if b >= nblocks:
                return b
        raise ValueError(f"sequence needs {nblocks} blocks > max {self.max_blocks}")

    def _run(self, header: np.ndarray, host_t: torch.Tensor) -> torch.Tensor:
        kind = "decode" if header[0] == KIND_DECODE else "prefill"
        T, nseq_l, max_blocks, ntiles, nseq, filt = (int(x) for x in header[1:HEADER_LEN])
        lay = _Layout(T, nseq_l, max_blocks, prefill=kind == "prefill", ntiles=ntiles)
        if self.use_graphs and (kind == "decode" or header[0] == KIND_PREFILL_GRAPH):
            if kind == "decode":
                key = (T, max_blocks, bool(filt))
                self.graph_replays += 1
            else:
                key = ("prefill", T, nseq_l, max_blocks, ntiles, bool(filt))
                self.prefill_graph_replays += 1
            g = self.graphs.get(key)
            if g is None:
                if kind == "decode":
                    self._capture(T, max_blocks, bool(filt))
                else:
                    self._capture(T, max_blocks, bool(filt), prefill=lay)
                g = self.graphs[key]
            graph, dev, out, exec_ = g
            if exec_:
                # H2D + hipGraphLaunch with the GIL held (torch's copy_ / replay() release it and the engine
                # thread then waits for the event-loop thread: csrc/bindings/torch_ops.cpp, graph_launch)
                nat = _native.ops()
                nat.copy_async(dev, host_t, lay.size * 4, self.device.index or 0)
                t_h2d = time.perf_counter()
                nat.graph_launch(exec_, self.device.index or 0)
                self.timing["graph_launch"] += time.perf_counter() - t_h2d
            else:
                dev.copy_(host_t[:lay.size], non_blocking=True)
                graph.replay()
            ids = out
        else:
            dev = self.model.ws.get("meta." + kind, (lay.size,), torch.int32, self.device)
            dev.copy_(host_t[:lay.size], non_blocking=True)
            fb = self._forward_batch(kind, lay, dev, nseq_l, filtered=bool(filt))
            ids = self.model.forward(fb, self.kv)
        return ids

    # ------------------------------------------------------------------------------------------
    def _capture(self, bucket: int, max_blocks: int, filtered: bool = False, prefill: _Layout | None = None) -> None:
        """Capture the decode forward for `bucket` rows and a `max_blocks`-wide block table, with or
        without the top-k / top-p resampler (largest first avoids workspace growth).  ``prefill``: capture
        that padded prefill layout instead (the warmup and capture run on all-padding metadata: no cache
        slot is written, every attention tile exits)."""
        lay = prefill if prefill is not None else _Layout(bucket, bucket, max_blocks, prefill=False)
        kind = "prefill" if prefill is not None else "decode"
        dev = torch.zeros(lay.size, dtype=torch.int32, device=self.device)
        host = self._host(lay.size, "capture")
        hn = host.numpy()
        self._fill(lay, hn, [], [])
        dev.copy_(host[:lay.size])
        fb = self._forward_batch(kind, lay, dev, lay.nseq, filtered=filtered)
        # eager warmup: allocates workspace and loads kernels outside the capture
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self.model.forward(fb, self.kv)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if self._graph_pool is None:
            self._graph_pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self._graph_pool):
            out = self.model.forward(fb, self.kv)
        torch.cuda.synchronize()
        exec_ = 0
        if _native.available() and os.environ.get("SYMMETRY_GRAPH_LAUNCH", "native") == "native":
            try:
                exec_ = int(g.raw_cuda_graph_exec())
            except Exception:  # noqa: BLE001 -- older torch: replay() it is
                exec_ = 0
        key = (bucket, max_blocks, filtered) if prefill is None else \
            ("prefill", lay.T, lay.nseq, lay.max_blocks, lay.ntiles, filtered)
        self.graphs[key] = (g, dev, out, exec_)

    def capture_all(self) -> float:
        """Rank 0: capture every (batch, context) decode graph; under TP each capture is mirrored by the
        workers (the graphs contain RCCL collectives, so all ranks must capture together)."""
        t0 = time.perf_counter()
        if self.use_graphs:
            for mb in sorted(self.ctx_blocks, reverse=True):
                for b in sorted(self.buckets, reverse=True):
                    if (b, mb, False) not in self.graphs:
                        if self.meta is not None:
                            self._broadcast(np.array([CMD_CAPTURE, b, b, mb, 0, b, 0], dtype=np.int32),
                                            torch.zeros(0, dtype=torch.int32))
                        self._capture(b, mb)
            if self._prefill_graphs_on():
                for mb in sorted(self.ctx_blocks, reverse=True):
                    for T in sorted((b for b in PREFILL_GRAPH_BUCKETS if b <= PREFILL_GRAPH_TOKENS), reverse=True):
                        for n in PREFILL_CAPTURE_SEQS:
                            lay = _Layout(T, n, mb, prefill=True, ntiles=self._pad_tiles(T, n))
                            if ("prefill", T, n, mb, lay.ntiles, False) not in self.graphs:
                                self._capture(T, mb, False, prefill=lay)
        return time.perf_counter() - t0

    # ------------------------------------------------------------------------------------------
    # tensor-parallel metadata plane (R4)
    def _broadcast(self, header: np.ndarray, host_t: torch.Tensor) -> None:
        self.meta.send(header, host_t.numpy() if host_t.numel() else None)

    def broadcast_stop(self) -> None:
        if self.tp_size > 1 and self.meta is not None and self.tp_rank == 0 and not self._stop_sent:
            self._stop_sent = True
            self.meta.send(np.array([CMD_STOP] + [0] * (HEADER_LEN - 1), dtype=np.int32), None)
            self.meta.close()

    def sync_point(self) -> float:
        """Every rank's GPU idle + a barrier over the bootstrap group; returns this rank's host time.  Under
        TP rank 0 sends CMD_SYNC so the workers (in :meth:`worker_loop`) meet it (bench timing brackets)."""
        import torch.distributed as dist

        if self.meta is not None and self.tp_rank == 0:
            self.meta.send(np.array([CMD_SYNC] + [0] * (HEADER_LEN - 1), dtype=np.int32), None)
        if self.is_gpu:
            torch.cuda.synchronize()
        if self.meta is not None:
            dist.barrier(group=self.cpu_group)
        if self.is_gpu:
            torch.cuda.synchronize()
        return time.perf_counter()

    WORKER_SLOTS = 4  # pinned metadata buffers a worker cycles through (H2D copies still in flight)

    def _worker_host(self, n: int) -> torch.Tensor:
        """A pinned buffer whose previous H2D copy (WORKER_SLOTS steps ago) has completed."""
        if not self._wslots:
            self._wslots = [[None, None] for _ in range(self.WORKER_SLOTS)]
        slot = self._wslots[self._wnext]
        self._wnext = (self._wnext + 1) % self.WORKER_SLOTS
        if slot[1] is not None:
            slot[1].synchronize()  # normally long done: the GPU is at most a step or two behind
        if slot[0] is None or slot[0].numel() < n:
            slot[0] = torch.empty(max(n, 1024), dtype=torch.int32, pin_memory=self.is_gpu)
        self._wslot = slot
        return slot[0][:n]

    def worker_loop(self) -> None:
        """Ranks 1..tp-1: mirror rank 0's steps until it sends stop.  Never synchronises the stream: the
        next step's metadata is popped and enqueued while the GPU still runs this one (the xGMI
        collectives keep the ranks in step on the device).  A collective that gave up waiting for a peer
        (the communicator's host-mapped error word) ends the worker with an error: its partial sums would
        be garbage."""
        try:
            self._worker_loop()
        except BaseException as exc:
            # tell rank 0 at once over the ring's back-channel (its health monitor fails the provider), then die
            code = 2 if isinstance(exc, KeyboardInterrupt) else 3
            try:
                self.meta.report(code)
            except Exception:  # noqa: BLE001
                pass
            raise

    def _worker_loop(self) -> None:
        check = getattr(self.model.tp, "error", None)
        while True:
            msg = self.meta.recv()
            if msg is None:
                return
            header, payload = msg
            if header[0] == CMD_STOP:
                return
            if header[0] == CMD_SYNC:
                self.sync_times.append(self.sync_point())
                continue
            n = int(payload.size)
            host_t = self._worker_host(max(n, 1))
            if n:
                host_t.numpy()[:n] = payload
            if header[0] == CMD_CAPTURE:
                self._capture(int(header[1]), int(header[3]), bool(header[6]))
                continue
            self._run(header[:HEADER_LEN], host_t)
            if self.is_gpu:
                ev = torch.cuda.Event()
                ev.record()
                self._wslot[1] = ev
            if not self.is_gpu:
                continue
            err = check() if check is not None else 0
            if err:
                from ..parallel.health import TPFaultError

                raise TPFaultError(f"TP rank {self.tp_rank}: xGMI collective gave up waiting for rank {err - 1}")
