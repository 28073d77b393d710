"""Engine: a batch of Splendor tables resident on one MI355X, driven through the C-ABI.

All buffers are PyTorch-ROCm tensors (caller-owned device memory, include/splendor_amd.h
"Conventions"); launches go on the current torch stream, so they compose with torch work and
never synchronise the host except for the explicit download/upload helpers.
"""
import ctypes

import numpy as np

from . import _native
from ._native import NUM_ACTIONS, OBS_DIM, OBS_U8, TABLE_DTYPE, ArenaDesc, LaunchFault, StepArgs, check, ptr
from .engine.state import load_tables
from .seeding import pcg64_states


class Engine:
    """`num_tables` independent tables of `num_players` players on `device`.

    table0: global id of table 0 — the policy stream of a shard is keyed by global table ids,
    so results do not depend on how tables are split across GPUs.
    refill_period / refill_fused: pool refill every `refill_period` steps; rollout() runs a due
    refill inside its launch unless refill_fused is False (results are the same either way).
    pipeline: rollout() kernel choice, same results in every mode: True = auto (the three-wave dealer
              variant for grids of at most two workgroups per CU, else two-wave at 64 tables per
              workgroup); "always" / "half" = two-wave at 64 / 32 tables per workgroup; "dealer" = the
              dealer variant; "dealer2" = the six-wave dealer variant (SIMD-aware roles); "quad" = four
              two-wave teams per workgroup, one workgroup per CU (SIMD-aware roles, partner hand-off);
              False = one wave per 64 tables.
    """

    # pool refill period by player count (three pool deals per table cover the resets in between;
    # random games last ~77 plies at 2p, ~29 at 4p)
    DEFAULT_REFILL = {2: 64, 3: 32, 4: 16}

    def __init__(self, num_tables, num_players=2, device=None, refill_period=None, table0=0, refill_fused=True,
                 pipeline=True, delegation=None, cards=None, partner_lead=None, host_io=False, step_tail=None):
        torch = _native.require_gpu()
        self.torch = torch
        self.lib = _native.load_library()
        if not 2 <= num_players <= 4:
            raise ValueError("num_players must be 2..4")
        if num_tables <= 0:
            raise ValueError("num_tables must be positive")
        self.n, self.P, self.table0 = int(num_tables), int(num_players), int(table0)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self._settings = (refill_period, refill_fused, pipeline, delegation, partner_lead)
        self._step_tail = step_tail
        self.ctx = None
        self._fault_carry = 0  # a fault seen on a context replaced by set_card_table
        self._create_ctx(cards)
        nbytes = int(self.lib.spl_arena_bytes(self.n, self.P))
        dev = self.device
        self._arena_raw = torch.zeros(nbytes + 256, dtype=torch.uint8, device=dev)
        off = (-self._arena_raw.data_ptr()) % 256
        self.arena = self._arena_raw[off:off + nbytes]
        self.desc = ArenaDesc(self.arena.data_ptr(), nbytes, self.n, self.P, 0, 0)
        self._step_args = {}  # cached spl_step argument blocks per output set (Engine.step)
        n = self.n
        # one contiguous I/O block: per-step outputs first (a single copy fetches a small batch)
        specs = [("obs", torch.int32, (n, OBS_DIM)), ("mask", torch.int8, (n, NUM_ACTIONS)),
                 ("reward", torch.float32, (n,)), ("terminated", torch.uint8, (n,)), ("flags", torch.uint8, (n,)),
                 ("winner", torch.int8, (n,)), ("actions", torch.int32, (n,)),
                 ("final_obs", torch.int32, (n, OBS_DIM))]
        offs, off = [], 0
        for name, dt, shape in specs:
            nb = int(np.prod(shape)) * torch.empty((), dtype=dt).element_size()
            offs.append((name, dt, shape, off, nb))
            off = (off + nb + 255) // 256 * 256
        # host_io (the single-table SplendorEnv): the I/O block lives in pinned host memory, which the
        # kernels read (actions) and write (outputs) through its device mapping — a step is then one
        # launch and a stream synchronisation, no fill kernel for the action and no copy of the outputs
        self.host_io = bool(host_io)
        self.io = (torch.zeros(off, dtype=torch.uint8, pin_memory=True) if self.host_io
                   else torch.zeros(off, dtype=torch.uint8, device=dev))
        if self.host_io and not self._host_mapped(self.io.data_ptr()):
            # the caching host allocator handed out memory the device does not see at the same address
            # (e.g. registered instead of allocated pinned memory): device I/O block instead;
            # SplendorEnv then copies the action in and the outputs out (host_io is False)
            self.host_io = False
            self.io = torch.zeros(off, dtype=torch.uint8, device=dev)
        for name, dt, shape, o, nb in offs:
            setattr(self, name, self.io[o:o + nb].view(dt).view(shape))
        self.io_step_bytes = offs[6][3]  # obs .. winner
        with torch.cuda.device(dev):
            check(self.lib, self.lib.spl_arena_init(self.ctx, ctypes.byref(self.desc), self.stream()))

    def _host_mapped(self, ptr):
        """Whether pinned host memory at `ptr` is mapped into the device at the same address
        (spl_host_mapped), so the kernels may be handed the host pointer itself."""
        same = ctypes.c_int32(0)
        check(self.lib, self.lib.spl_host_mapped(ctypes.c_void_p(ptr), ctypes.byref(same)))
        return bool(same.value)

    def _create_ctx(self, cards=None):
        """A library context over the card table `cards` (int32 [90, 8]; None = the canonical
        engine/data/tables.json) and the canonical nobles, with this engine's settings."""
        torch = self.torch
        base_cards, nobles = load_tables()
        tbl = base_cards if cards is None else np.ascontiguousarray(np.asarray(cards, np.int32))
        if tbl.shape != (90, 8):
            raise ValueError("card table must be int32 [90, 8]")
        ctx = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_ctx_create(self.device.index, tbl.ctypes.data, nobles.ctypes.data,
                                                    ctypes.byref(ctx)))
        self.ctx = ctx
        # the context's fault word (host-mapped; the kernels write a faulting launch's serial there)
        self._fault_word = ctypes.c_uint64.from_address(self.lib.spl_ctx_fault_word(ctx))
        self.custom_cards = None if cards is None else tbl.copy()
        refill_period, refill_fused, pipeline, delegation, partner_lead = self._settings
        num_players = self.P
        if refill_period is None:
            refill_period = self.DEFAULT_REFILL.get(int(num_players), 16)
        check(self.lib, self.lib.spl_ctx_set_refill_period(self.ctx, int(refill_period)))
        # rollout(): a due refill runs inside the rollout launch (True) or as a refill launch after it
        check(self.lib, self.lib.spl_ctx_set_refill_fused(self.ctx, 1 if refill_fused else 0))
        # rollout(): two-wave pipelined kernel or one wave per 64 tables; same results
        pipe = {"always": 2, "half": 3, "dealer": 4, "dealer2": 5, "quad": 6}.get(pipeline, 1 if pipeline else 0)
        check(self.lib, self.lib.spl_ctx_set_rollout_pipeline(self.ctx, pipe))
        # rollout() into a per-step store: every n-th step the odd-XCC workgroups' rows are stored by
        # their even-XCC partners (None = the library default, 0 = off); same results
        if delegation is not None:
            check(self.lib, self.lib.spl_ctx_set_rollout_delegation(self.ctx, int(delegation)))
        # rollout() of the six-wave dealer into a per-step store: a team this many steps behind its
        # neighbouring-XCC partner hands it whole steps of rows (None = library default, 0 = off,
        # -1 = whenever a slot is free); same results
        if partner_lead is not None:
            check(self.lib, self.lib.spl_ctx_set_partner_lead(self.ctx, int(partner_lead)))
        # step(): three waves per 64 tables (a tail wave takes the legal mask off the rules wave) or two;
        # None = the library's choice by grid size (spl_ctx_set_step_tail); same results
        if self._step_tail is not None:
            check(self.lib, self.lib.spl_ctx_set_step_tail(self.ctx, int(self._step_tail)))

    def set_card_table(self, cards=None):
        """Evaluate the tables from now on with card table `cards` (int32 [90, 8]; None = canonical):
        a new context over the same arena (the table state does not depend on the context)."""
        same = (cards is None and self.custom_cards is None) or (
            cards is not None and self.custom_cards is not None and np.array_equal(cards, self.custom_cards))
        if same:
            return
        self.torch.cuda.synchronize(self.device)
        old = self.ctx
        self._fault_carry = self.faults()
        self._create_ctx(cards)
        self.lib.spl_ctx_destroy(old)

    # ------------------------------------------------------------------------------------
    def faults(self):
        """Serial of a launch that faulted since the last clear_faults() (0 = none): a lost internal
        hand-off in a dealer-variant rollout (include/splendor_amd.h spl_ctx_faults).  Reads the
        host-mapped fault word: no synchronisation, covers every launch that has finished."""
        if self._fault_word is None:  # closed: the word was freed with the context
            return self._fault_carry
        return self._fault_carry or int(self._fault_word.value)

    def check_faults(self):
        """Raise LaunchFault if a launch of this engine faulted (no synchronisation); RuntimeError
        once the engine is closed (its context and fault word are gone)."""
        if self.ctx is None:
            raise RuntimeError("splendor engine: used after close()")
        f = self.faults()
        if f:
            raise LaunchFault(f"splendor engine: launch {f} lost an internal hand-off; its outputs from the faulted "
                              "step on are not written (flags carry SPL_F_FAULT) and the tables' state is undefined: "
                              "reset the tables, then clear_faults()")

    def clear_faults(self):
        """Wait for this engine's work, then zero its fault word."""
        self.torch.cuda.synchronize(self.device)
        self._fault_carry = 0
        f = ctypes.c_uint64()
        check(self.lib, self.lib.spl_ctx_faults(self.ctx, ctypes.byref(f), 1))

    def stream(self):
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "ctx", None) is not None and self.ctx.value:
            self.torch.cuda.synchronize(self.device)
            self._fault_carry = self.faults()  # kept readable after the word is freed
            self._fault_word = None
            self.lib.spl_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------------------------
    def reset(self, seeds=None, mask=None, obs=True, obs_out=None, mask_out=None):
        """Reset tables (all, or where `mask` is true).  seeds: None continues every table's
        engine-seed stream (reset() without a seed); else one seed per table (reset(seed=s)).
        Writes every table's observation / action mask to obs_out / mask_out (default self.obs /
        self.mask; obs=False writes neither)."""
        torch = self.torch
        pcg = None
        if seeds is not None:
            seeds = list(seeds)
            if len(seeds) != self.n:
                raise ValueError(f"expected {self.n} seeds")
            pcg = torch.from_numpy(pcg64_states(seeds).reshape(-1)).to(self.device)
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
            if m.numel() != self.n:
                raise ValueError("mask must have one entry per table")
        with torch.cuda.device(self.device):
            o = (self.obs if obs_out is None else obs_out) if obs else None
            mk = (self.mask if mask_out is None else mask_out) if obs else None
            check(self.lib, self.lib.spl_reset(self.ctx, ctypes.byref(self.desc), ptr(pcg), ptr(m), ptr(o), ptr(mk),
                                               self.stream()))
        self._keep = (pcg, m)  # alive until the async reset has consumed them
        return o, mk

    def deal(self, engine_seeds, mask=None, obs=True):
        """initial_state(P, seed) for every table (or where `mask` is true) from explicit engine
        seeds (engine/state.py:181-211; CPython seeds are taken by absolute value, < 2**32)."""
        torch = self.torch
        seeds = np.asarray([abs(int(x)) for x in engine_seeds], dtype=np.uint64)
        if len(seeds) != self.n:
            raise ValueError(f"expected {self.n} engine seeds")
        if (seeds >= 2**32).any():
            raise ValueError("engine seeds must satisfy abs(seed) < 2**32 on the device")
        es = torch.from_numpy(seeds.astype(np.uint32)).to(self.device)
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        with torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_deal(self.ctx, ctypes.byref(self.desc), ptr(es), ptr(m),
                                              ptr(self.obs) if obs else None, ptr(self.mask) if obs else None,
                                              self.stream()))
        self._keep = (es, m)
        return self.obs, self.mask

    def step(self, actions=None, autoreset=True, final_obs=True, next_actions=None, policy_seed=0, ply=0,
             ep_return=None, ep_count=None, ply_base=None, policy=0, small=None, obs_u8=None, gate=None,
             keep_obs=False):
        """One env step on every table (SplendorEnv.step semantics per table).  autoreset: False,
        True (same-step autoreset) or 2 (also re-deal tables terminal on entry, without a move).
        next_actions (optional int32 tensor) receives `policy`'s action (_native.POLICY_*) over
        the new state.  small: optional (reward, terminated, flags, winner) tensors that receive
        those outputs instead of self.reward/terminated/flags/winner.  obs_u8: optional uint8
        [n, 300] tensor that receives the compact observation (spl_step_args_t.obs_u8) INSTEAD of
        self.obs (a device policy's input at a quarter of the bytes; self.obs is left as it was), or with
        keep_obs=True beside it (self.obs written as usual, obs_u8 a copy of its rows; ABI 8).
        gate: optional (terminated, flags) uint8 tensors of the agent's move in a dual step — tables
        where it ended the game or was not applied get action -1 (written into `actions`) and are not
        moved (spl_step_args_t.gate_*; spl_dual_gate fused into this launch)."""
        torch = self.torch
        if self.ctx is None:
            raise RuntimeError("splendor engine: used after close()")
        if actions is None:
            actions = self.actions
        if not (isinstance(actions, torch.Tensor) and actions.dtype == torch.int32 and actions.is_contiguous()
                and (actions.device == self.device or (self.host_io and actions is self.actions))):
            actions = torch.as_tensor(actions, device=self.device).to(torch.int32).contiguous()
        if actions.numel() != self.n:
            raise ValueError(f"expected {self.n} actions")
        rw, tm, fl, wn = small if small is not None else (self.reward, self.terminated, self.flags, self.winner)
        code = (2 if autoreset == 2 else 1) if autoreset else 0
        fo = bool(final_obs and autoreset)
        # the argument block of this output set is built once; per call only the inputs change
        if obs_u8 is not None and not (obs_u8.device == self.device and obs_u8.dtype == torch.uint8
                                       and obs_u8.is_contiguous() and obs_u8.numel() == self.n * OBS_U8):
            raise ValueError(f"obs_u8 must be a contiguous uint8 [{self.n}, {OBS_U8}] tensor on {self.device}")
        u8 = None if obs_u8 is None else obs_u8.data_ptr()
        both = bool(keep_obs and u8)
        key = (rw.data_ptr(), tm.data_ptr(), fl.data_ptr(), wn.data_ptr(), code, fo, u8, both)
        a = self._step_args.get(key)
        if a is None:
            a = StepArgs(obs=None if (u8 and not both) else self.obs.data_ptr(), obs_u8=u8, mask=self.mask.data_ptr(),
                         reward=rw.data_ptr(), terminated=tm.data_ptr(), flags=fl.data_ptr(), winner=wn.data_ptr(),
                         final_obs=self.final_obs.data_ptr() if fo else None, autoreset=code, table0=self.table0)
            if len(self._step_args) >= 16:  # callers that pass fresh output tensors every call
                self._step_args.clear()
            self._step_args[key] = a
        a.actions = actions.data_ptr()
        a.policy = int(policy)
        a.next_actions = None if next_actions is None else next_actions.data_ptr()
        a.ply_base = None if ply_base is None else ply_base.data_ptr()
        a.policy_seed = int(policy_seed) & (2**64 - 1)
        a.ply = int(ply) & (2**64 - 1)
        a.ep_return = None if ep_return is None else ep_return.data_ptr()
        a.ep_count = None if ep_count is None else ep_count.data_ptr()
        a.gate_terminated = None if gate is None else gate[0].data_ptr()
        a.gate_flags = None if gate is None else gate[1].data_ptr()
        if torch.cuda.current_device() == self.device.index:
            check(self.lib, self.lib.spl_step(self.ctx, ctypes.byref(self.desc), ctypes.byref(a), self.stream()))
        else:
            with torch.cuda.device(self.device):
                check(self.lib, self.lib.spl_step(self.ctx, ctypes.byref(self.desc), ctypes.byref(a), self.stream()))
        self._keep_actions = actions
        return self.obs, self.mask, rw, tm, fl

    def host_stepper(self):
        """SplendorEnv's per-call path: a launcher of spl_step over this engine's own actions and
        outputs, autoreset off, no policy (what step(self.actions, autoreset=False) launches), with the
        argument block built once — the per-call Python of step() is most of a one-table step's time."""
        torch, lib, dev, idx = self.torch, self.lib, self.device, self.device.index
        a = StepArgs(actions=self.actions.data_ptr(), obs=self.obs.data_ptr(), mask=self.mask.data_ptr(),
                     reward=self.reward.data_ptr(), terminated=self.terminated.data_ptr(), flags=self.flags.data_ptr(),
                     winner=self.winner.data_ptr(), final_obs=None, autoreset=0, table0=self.table0)
        ref = ctypes.byref(a)

        def go():
            if self.ctx is None:
                raise RuntimeError("splendor engine: used after close()")
            s = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            if torch.cuda.current_device() == idx:
                rc = lib.spl_step(self.ctx, ctypes.byref(self.desc), ref, s)
            else:
                with torch.cuda.device(dev):
                    rc = lib.spl_step(self.ctx, ctypes.byref(self.desc), ref, s)
            if rc:
                check(lib, rc)
        go.args = a  # the block the launches point at
        return go

    def rollout(self, steps, actions=None, next_actions=None, policy_seed=0, ply=0, out=None, final_obs=True,
                ep_return=None, ep_count=None, ply_base=None, policy=0):
        """`steps` env steps of every table under the device uniform-random policy in one launch
        (spl_rollout): the same trajectory as `steps` calls of step() with next_actions fed back
        and ply, ply+1, ...  out=None overwrites self.obs/mask/... each step; otherwise `out` is a
        dict of [steps, n, ...] tensors (obs, mask, reward, terminated, flags, winner, final_obs)
        that receives every step's outputs (rollout storage).  Raises LaunchFault when an earlier
        launch faulted (check_faults; a rollout's own fault shows at the next call or check)."""
        self.check_faults()
        torch = self.torch
        actions = self.actions if actions is None else actions
        if not (isinstance(actions, torch.Tensor) and actions.device == self.device and actions.dtype == torch.int32
                and actions.is_contiguous() and actions.numel() == self.n):
            raise ValueError("actions must be a contiguous int32 device tensor with one entry per table")
        if out is None:
            bufs, per_step = dict(obs=self.obs, mask=self.mask, reward=self.reward, terminated=self.terminated,
                                  flags=self.flags, winner=self.winner, final_obs=self.final_obs), 0
        else:
            bufs, per_step = out, 1
            for k, shape in (("obs", (steps, self.n, OBS_DIM)), ("mask", (steps, self.n, NUM_ACTIONS)),
                             ("reward", (steps, self.n)), ("terminated", (steps, self.n)), ("flags", (steps, self.n))):
                if k not in bufs or tuple(bufs[k].shape) != shape or not bufs[k].is_contiguous():
                    raise ValueError(f"out[{k!r}] must be a contiguous tensor of shape {shape}")
        a = StepArgs(actions=actions.data_ptr(), obs=bufs["obs"].data_ptr(), mask=bufs["mask"].data_ptr(),
                     reward=bufs["reward"].data_ptr(), terminated=bufs["terminated"].data_ptr(),
                     flags=bufs["flags"].data_ptr(), winner=ptr(bufs.get("winner")),
                     final_obs=ptr(bufs.get("final_obs")) if final_obs else None, autoreset=1, policy=int(policy),
                     next_actions=None if next_actions is None else next_actions.data_ptr(),
                     ply_base=None if ply_base is None else ply_base.data_ptr(),
                     policy_seed=int(policy_seed) & (2**64 - 1), ply=int(ply) & (2**64 - 1), table0=self.table0,
                     ep_return=None if ep_return is None else ep_return.data_ptr(),
                     ep_count=None if ep_count is None else ep_count.data_ptr())
        with torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_rollout(self.ctx, ctypes.byref(self.desc), ctypes.byref(a), int(steps),
                                                 per_step, self.stream()))
        self._keep_actions = (actions, bufs)
        return bufs

    def rollout_kernel_name(self, per_step=True):
        """Name of the kernel rollout() launches for this engine (as a rocprofv3 summary lists it)."""
        name = self.lib.spl_rollout_kernel_name(self.ctx, self.n, self.P, 1 if per_step else 0)
        if name is None:
            check(self.lib, -1)
        return name.decode()

    def refill(self):
        with self.torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_refill(self.ctx, ctypes.byref(self.desc), self.stream()))

    def encode(self, out=None):
        out = self.obs if out is None else out
        with self.torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_encode(self.ctx, ctypes.byref(self.desc), ptr(out), self.stream()))
        return out

    def legal(self, out=None):
        out = self.mask if out is None else out
        with self.torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_legal(self.ctx, ctypes.byref(self.desc), ptr(out), self.stream()))
        return out

    def sample_uniform(self, mask=None, out=None, seed=0, ply=0):
        mask = self.mask if mask is None else mask
        out = self.actions if out is None else out
        with self.torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_sample_uniform(self.ctx, self.n, ptr(mask), ptr(out), int(seed), int(ply),
                                                        self.table0, self.stream()))
        return out

    # ------------------------------------------------------------------------------------
    def download(self, first=0, count=None):
        """numpy TABLE_DTYPE[count] host views (synchronous; raises LaunchFault after a faulted launch)."""
        count = self.n - first if count is None else count
        out = np.zeros(count, TABLE_DTYPE)
        with self.torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_table_download(self.ctx, ctypes.byref(self.desc), first, count,
                                                        out.ctypes.data, self.stream()))
        self.check_faults()
        return out

    def upload(self, records, first=0):
        recs = np.ascontiguousarray(np.atleast_1d(records).astype(TABLE_DTYPE))
        with self.torch.cuda.device(self.device):
            check(self.lib, self.lib.spl_table_upload(self.ctx, ctypes.byref(self.desc), first, len(recs),
                                                      recs.ctypes.data, self.stream()))

    def token_lut(self):
        words = int(self.lib.spl_ctx_token_lut(self.ctx, None, 0))
        out = np.zeros(words, np.uint32)
        check(self.lib, self.lib.spl_ctx_token_lut(self.ctx, out.ctypes.data, words))
        return out.reshape(-1, 4)
