#!/usr/bin/env python3
"""Generator of the wave-tile pass kernel in gfx950 assembly (fp64 or fp32).

Why assembly: the kernel keeps a 2^(R+6)-amplitude tile in VGPRs across a
runtime-dispatched list of ops.  Written in HIP C++, LLVM's structurizer and
register allocator turned every dispatch arm into copies of the whole tile
(hundreds of v_mov per op, spills at any occupancy).  Here the tile lives in
FIXED registers for the whole kernel and every op handler updates it in
place; the host plan (src/core/wave.hpp) picks the handler of each op, whose
byte offset from the dispatch anchor is stored in the op record, and the
kernel jumps there with s_setpc_b64.

    python tools/gen_wave_asm.py asm   --prec 2 --slots 4 --out build/wave_f64/wave_kernel.s
    python tools/gen_wave_asm.py embed --prec 2 --obj build/wave_f64/wave_kernel.o \
        --hsaco build/wave_f64/wave_kernel.hsaco --out build/wave_f64/wave_image.inc

fp64 (--prec 2): a value is a VGPR pair, 2 values per 16-byte vector (tile
bit 0 in slot 0).  fp32 (--prec 1, the reference's QuEST_PREC=1 build,
QuEST_precision.h:17-62): one VGPR per value, 4 per vector (tile bits 0-1 in
slots 0-1) and 32 amplitudes per lane (--slots 5): the same registers and
bytes per tile, twice the amplitudes, full-rate fp32 arithmetic.

Register plan (R = slots, NS = 2^R amplitudes per lane, P = dwords per value):
    v[Pj : Pj+P-1]            re of register j        (j < NS)
    v[P NS + Pj ...]          im of register j
    T0..T15 (16 values)       temporaries;  C0, C1 per-lane coefficients
    vLane / vLdB / vStB       lane id, per-lane load / store byte offsets
Device records (host side: src/hip/backend_hip.hip, WaveLaunchDev / WaveOpDev):
    launch + 0    u64 numTiles          + 8   u64 waveStride
           + 16   u32 nOps              + 24  u32 pos[16]
           + 88   u64 ldGroupByte[16]   + 216 u64 stGroupByte[16]
           + 344  u32 ldLaneByte[64]    + 600 u32 stLaneByte[64]
           + 1024 u64 ldWaveByte[16]    + 1152 u64 stWaveByte[16]
           + 1280 u64 debugBuf       + 1288 u32 tileCounter[8]
           pos[b] for b >= 12 sits in bits 8.. of pos[b - 12]
           + 2048 WaveOpDev ops[]  (96 B: i32 handler, u32 cReg, u32 cLane,
                  u32 aux, u64 ctrlOut, u64 pad, f64 m[8] / f32 m[16])
Semantics of every op: src/core/wave.hpp (and the CPU emulation in
src/cpu/backend_cpu.cpp applyWaveOp, which the tests compare against).
"""
import argparse
import re
import struct
import sys

KINDS = ["M2", "M2R", "M2RI", "ANTI", "SWAP"]
LD_WAVE, ST_WAVE, DEBUG_BUF, OPS_OFF = 1024, 1152, 1280, 2048   # launch-record offsets (see above)
# dynamic tile claims of looping grids: u32 counters (one per launch sharing
# the record, kernel argument bits 5-7), zeroed by the host's upload
TILE_CNT = 1288
import os as _os
# cache policy of the state stream (non-temporal by default); WAVE_LD_POLICY /
# WAVE_ST_POLICY override for experiments, e.g. "" or " sc1"
LD_POLICY = _os.environ.get("WAVE_LD_POLICY", " nt")
ST_POLICY = _os.environ.get("WAVE_ST_POLICY", " nt")
# ---- handler table (shared with the host through wave_image.inc) ---------
# gates on lane bits 0-2 directly (no transposition)
LANE_KINDS, LANE_BITS = ["M2R", "M2RI", "ANTI", "SWAP"], 3
# cheaper forms of common gates (slot targets): shear rotations (Ry, Rx),
# the unnormalised Hadamard (its 1/sqrt2 is absorbed by another op of the
# pass, see src/core/wave.cpp) and Y / -Y as register swaps plus sign flips
KINDS2 = ["ROTY", "ROTX", "HADD", "YSW", "YSWC"]
# unit-modulus phases on the registers j with (j & creg) == creg (lane = 1:
# only on lanes whose cLane bits are set): rotation of (re, im) by three
# shears, negation, multiplication by +-i, negation + rotation
PH_KINDS = ["DROT", "DNEG", "DMULI", "DMULNI", "DROTN", "DSC"]   # DSC: real scale m[0] (dephasing factors)
# one-qubit density-matrix channels: a real superoperator on the 4-group of
# slots (a, b) = (row bit, column bit), g = bit a + 2 bit b: CH1 mixes
# (x0, x3) by a real 2x2 (m0 m1 / m2 m3) and scales x1, x2 by m4 (dephasing,
# depolarising, amplitude damping, density collapse); CHD only scales x1, x2
CH_KINDS = ["CH1", "CHD"]

# fp32 packed math (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32 on registers j,
# j + 1 held as one 64-bit pair): WAVE_PK=0 keeps scalar fp32 code
PK = _os.environ.get("WAVE_PK", "1") == "1"


def pk_fix(line):
    """Operand modifiers of a packed fp32 instruction written like its scalar
    form: v[a:b] pairs pass through (lo -> lo, hi -> hi); S<k> is the op
    record's coefficient s(76 + k) and B<r> the VGPR r, each broadcast to both
    halves (op_sel / op_sel_hi pick the dword of the aligned 64-bit pair);
    inline constants are broadcast; a leading '-' becomes neg_lo / neg_hi."""
    op, _, rest = line.partition(" ")
    ops = [x.strip() for x in rest.split(",")]
    dst, srcs = ops[0], ops[1:]
    out, sel, selhi, neg = [], [], [], []
    for x in srcs:
        n = x.startswith("-")
        if n:
            x = x[1:]
        m = re.fullmatch(r"([SB])(\d+)", x)
        if m:
            r = int(m.group(2)) + (76 if m.group(1) == "S" else 0)
            base, h = r & ~1, r & 1
            out.append(f"{'s' if m.group(1) == 'S' else 'v'}[{base}:{base + 1}]")
            sel.append(h)
            selhi.append(h)
        elif x.startswith("v["):
            out.append(x)
            sel.append(0)
            selhi.append(1)
        else:
            out.append(x)
            sel.append(0)
            selhi.append(0)
        neg.append(1 if n else 0)
    f = lambda v: "[" + ",".join(map(str, v)) + "]"
    s = f"{op} {dst}, " + ", ".join(out) + f" op_sel:{f(sel)} op_sel_hi:{f(selhi)}"
    if any(neg):
        s += f" neg_lo:{f(neg)} neg_hi:{f(neg)}"
    return s


LAYOUT = {}
SWAP64 = _os.environ.get("WAVE_SWAP64", "1") == "1"   # register exchanges as 64-bit moves (swap_vals)
# X / CNOT on lane bit 2 (LSWAP) through the LDS crossbar: one ds_swizzle_b32
# per dword (lane ^ 4) instead of two bank-masked DPP moves plus a 64-bit copy
# per value -- 320 VALU instructions per handler moved off the VALU, which the
# op-heavy passes are bound by (tools/experiments/valu_rate.hip: ds_swizzle
# issues at 1.5x an fp64 op per SIMD on the LDS pipe).  WAVE_SWZ=2: lane bits
# 0 and 1 too (their DPP version is 128 VALU; bench 0.1277 vs 0.1279 with
# lane bit 2 only vs 0.1289 ms/gate without, three rounds on one box), 3: the
# partner fetches of the lane-bit gates (LM2R / LM2RI / LANTI) as well, 0: DPP
# only.
SWZ = int(_os.environ.get("WAVE_SWZ", "2"))
# per-lane selects: v_cmp_*_e64 into this SGPR pair + v_cndmask_b32_e64 (a
# v_cndmask_b32_e32 reading vcc issues ~5x slower on gfx950, tools/isa_micro.hip)
SEL = "s[98:99]"
# lane transpositions through LDS for lane bits < WAVE_TR_LDS (default 0:
# DPP / v_permlane*_swap for all; through LDS measured slower, 0.139 ->
# 0.146-0.163 ms / gate for lane bits 0 / 0-1 / 0-3, profiles/r3/tr_lds_ab.txt)
TR_LDS = int(_os.environ.get("WAVE_TR_LDS", "0"))
# s_nop 3 pads after every tile load: the loads' issue paced (bench -0.4 %
# with one, neutral with three, profiles/r5/load_pacing_ab.txt; issuing them
# back to back -- the re / im bases hoisted out of the per-group address adds
# -- was 1.3 % slower, group_base_hoist_ab.txt)
LD_PACE = int(_os.environ.get("WAVE_LD_PACE", "1"))
# lane-control exec masks: s_mov_b64 exec straight after the v_cmp that writes
# its SGPR pair (no s_nop: SALU reads of VALU-written SGPRs are interlocked;
# WAVE_EXEC_NOP=1 restores the pad)
NOP_FREE_EXEC = _os.environ.get("WAVE_EXEC_NOP", "0") != "1"


# op record fields live in s[36:51] (prefetch buffer: record bytes 0-63) and
# s[68:91] (the running handler's copy; bytes 64-95 loaded by the handlers
# that read them): handler, cReg, cLane, aux, ctrlOut (2), cWave,
# cWaveZero, m[8] (fp64) / m[16] (fp32)
REC_LO, REC_HI = 68, 91


def set_layout(R):
    """Base index of every handler family for R register slots; the last
    entry ("done") is the end-of-list sentinel (the store epilogue)."""
    NS = 1 << R
    sizes = [("slot", len(KINDS) * 2 * R), ("d2s", 2 * R), ("d2l", 2), ("tr", 6 * R), ("diag", 2 * NS),
             ("trw", 4 * R), ("lane", 8 * len(LANE_KINDS)), ("slot2", len(KINDS2) * 2 * R),
             ("ph", len(PH_KINDS) * 2 * NS), ("ch", len(CH_KINDS) * R * R),
             # controls on lane bits only (cReg 0): exec set once, no per-register tests
             ("slotL", len(KINDS) * R), ("slot2L", len(KINDS2) * R), ("d2sL", R),
             # X on slot s / lane bit l with ONE slot control c of polarity v
             # (CNOTs): the registers fixed at generation time, no per-register tests
             ("swk", R * R * 2 + LANE_BITS * R * 2),
             # the shared check path of ops with tile / wave predicates
             ("check", 1)]
    LAYOUT.clear()
    LAYOUT["R"] = R
    i = 0
    for name, n in sizes:
        LAYOUT[name] = i
        i += n
    LAYOUT["done"] = i


def idx_slot(kind, s, ctrl):
    if ctrl == 2:
        return LAYOUT["slotL"] + KINDS.index(kind) * LAYOUT["R"] + s
    return LAYOUT["slot"] + KINDS.index(kind) * 2 * LAYOUT["R"] + s * 2 + ctrl


def idx_swk(lane, t, c, v):
    """X on slot t (lane = 0) or lane bit t (lane = 1) controlled by slot c
    being v."""
    R = LAYOUT["R"]
    return LAYOUT["swk"] + (R * R * 2 if lane else 0) + (t * R + c) * 2 + v


def idx_d2s(s, ctrl):
    if ctrl == 2:
        return LAYOUT["d2sL"] + s
    return LAYOUT["d2s"] + s * 2 + ctrl


def idx_d2l(ctrl):
    return LAYOUT["d2l"] + ctrl


def idx_tr(s, l):
    return LAYOUT["tr"] + s * 6 + l


def idx_diag(creg, lane):
    return LAYOUT["diag"] + creg * 2 + lane


def idx_trw(s, b):
    return LAYOUT["trw"] + s * 4 + b


def idx_lane(kind, l, ctrl):
    return LAYOUT["lane"] + LANE_KINDS.index(kind) * 8 + l * 2 + ctrl


def idx_slot2(kind, s, ctrl):
    if ctrl == 2:
        return LAYOUT["slot2L"] + KINDS2.index(kind) * LAYOUT["R"] + s
    return LAYOUT["slot2"] + KINDS2.index(kind) * 2 * LAYOUT["R"] + s * 2 + ctrl


def idx_ph(kind, creg, lane):
    return LAYOUT["ph"] + PH_KINDS.index(kind) * 2 * (1 << LAYOUT["R"]) + creg * 2 + lane


def idx_ch(kind, a, b):
    return LAYOUT["ch"] + CH_KINDS.index(kind) * LAYOUT["R"] ** 2 + a * LAYOUT["R"] + b


def table_size(R):
    set_layout(R)
    return LAYOUT["done"] + 1


_VREG = re.compile(r"v\[(\d+):(\d+)\]|\bv(\d+)\b|\b(vcc)\b|(s\[98:99\])")


def _regs(operand):
    out = set()
    for m in _VREG.finditer(operand):
        if m.group(1):
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
        elif m.group(3):
            out.add(int(m.group(3)))
        elif m.group(4):
            out.add("vcc")
        else:
            out.add("sel")   # the SEL mask pair
    return out


def schedule(body):
    """List-schedule a straight-line VALU region: keep every RAW / WAR / WAW
    order of the program, otherwise issue the longest-critical-path
    instruction whose operands are ready (fp64 results assumed ready 3 issue
    slots later, others 2) -- interleaves the independent FMA chains of
    different pairs / elements instead of stalling on each chain."""
    n = len(body)
    defs, uses, lat = [], [], []
    for ins in body:
        op, _, rest = ins.partition(" ")
        ops = [x.strip() for x in rest.split(",")] if rest else []
        d = _regs(ops[0]) if ops else set()
        u = set()
        for x in ops[1:]:
            u |= _regs(x)
        if op.startswith("v_swap"):
            u |= d | _regs(ops[1])
            d = d | _regs(ops[1])
        if op.startswith("v_cndmask_b32_e32"):
            u.add("vcc")
        if op.startswith("v_fmac"):
            u |= d
        defs.append(d)
        uses.append(u)
        lat.append(3 if "f64" in op else 2)
    preds = [dict() for _ in range(n)]   # pred -> delay
    last_w, readers = {}, {}
    for i in range(n):
        for r in uses[i]:
            if r in last_w:
                w = last_w[r]
                preds[i][w] = max(preds[i].get(w, 0), lat[w])
        for r in defs[i]:
            for rd in readers.get(r, ()):
                if rd != i:
                    preds[i][rd] = max(preds[i].get(rd, 0), 1)
            if r in last_w and last_w[r] != i:
                preds[i][last_w[r]] = max(preds[i].get(last_w[r], 0), 1)
        for r in uses[i]:
            readers.setdefault(r, []).append(i)
        for r in defs[i]:
            last_w[r] = i
            readers[r] = []
    succs = [[] for _ in range(n)]
    for i in range(n):
        for p in preds[i]:
            succs[p].append(i)
    crit = [0] * n
    for i in range(n - 1, -1, -1):
        crit[i] = lat[i] + max((crit[s] for s in succs[i]), default=0)
    done = [False] * n
    at = [0] * n
    left = [len(preds[i]) for i in range(n)]
    ready = [i for i in range(n) if left[i] == 0]
    out, t = [], 0
    while ready:
        def earliest(i):
            return max((at[p] + d for p, d in preds[i].items()), default=0)
        avail = [i for i in ready if earliest(i) <= t]
        if not avail:
            t = min(earliest(i) for i in ready)
            continue
        i = max(avail, key=lambda k: (crit[k], -k))
        ready.remove(i)
        done[i] = True
        at[i] = t
        out.append(body[i])
        t += 1
        for s2 in succs[i]:
            left[s2] -= 1
            if left[s2] == 0:
                ready.append(s2)
    assert len(out) == n
    return out


class Gen:
    def __init__(self, R, dbuf, W, P=2, debug=False, nomem=False, lean=False, pfa=0, pfl=0):
        self.lean = lean        # 80 VGPRs / half outboxes: three 8-wave workgroups per CU
        self.nomem = nomem      # experiment: no state loads / stores (compute time alone)
        self.debug = debug
        self.R = R
        self.NS = 1 << R
        self.P = P               # dwords per value: 2 fp64, 1 fp32
        self.F = "f64" if P == 2 else "f32"
        self.MOV = "v_mov_b64" if P == 2 else "v_mov_b32"
        self.VB = 1 if P == 2 else 2   # tile bits inside one 16-byte vector (slots 0..VB-1)
        self.dbuf = dbuf
        self.W = W               # wave bits: 2^W waves share a tile (LDS exchanges)
        self.NW = 1 << W
        # bytes of one wave's LDS outbox (NS values x 64 lanes; lean: half of
        # them, a wave-bit transposition then runs in two rounds)
        self.OUTBOX = self.NS * 64 * 4 * P // (2 if lean else 1)
        self.lines = []
        # v[0 : 2P NS) the tile being processed (A), then the next tile being
        # loaded (B, software pipeline; dbuf only), then temporaries
        self.B = 2 * P * self.NS if dbuf else 0
        D = (2 if dbuf else 1) * 2 * P * self.NS
        self.D = D
        if not lean:
            # 16 temporaries (values): pairs / elements of a handler cycle
            # through 4 / 8 sets so that the scheduler can interleave them
            self.NT = 16
            self.T = [D + P * k for k in range(16)]
            self.C0, self.C1 = D + 16 * P, D + 17 * P
            self.vLane, self.vLdB, self.vStB, self.vTmp = D + 18 * P, D + 18 * P + 1, D + 18 * P + 2, D + 18 * P + 3
            self.CL = D + 18 * P + 4       # 4 values: per-lane coefficients of the lane-bit gates
            self.CLA = self.CL + 2 * P     # the anti-diagonal's pair of them
            self.nvgpr = D + 22 * P + 4    # fp64 R = 4: 112 VGPRs, 4 waves per SIMD
        else:
            # 4 temporaries (every set index aliases them: the scheduler keeps
            # the order), the lane-gate coefficients in temporaries 2-3, the
            # lane gates one amplitude at a time: fp64 80 VGPRs, 6 waves per SIMD
            # fp32 with packed math: 8 temporaries (four 64-bit pairs), C0 even
            nt = 8 if (P == 1 and PK) else 4
            self.NT = nt
            self.T = [D + P * (k % nt) for k in range(16)]
            self.C0, self.C1 = D + nt * P, D + (nt + 1) * P
            self.vLane, self.vLdB, self.vStB, self.vTmp = (D + (nt + 2) * P, D + (nt + 2) * P + 1,
                                                           D + (nt + 2) * P + 2, D + (nt + 2) * P + 3)
            self.CL = self.C0             # lane-gate coefficients in C0 / C1 (scratch: vTmp)
            self.CLA = self.C0
            self.nvgpr = D + (nt + 2) * P + 4
        # dynamic tile claims (looping grids): the claimed counter value (wave 0,
        # lane 0) and the LDS address of the slot it is published through
        self.vNext, self.vSlot = self.nvgpr, self.nvgpr + 1
        self.nvgpr += 2
        # next-tile prefetch of looping grids (pf_paths): PFA of a tile's
        # 16-byte loads per lane land in AGPRs, PFL in this wave's LDS area
        # (vPF: its address for this lane); the rest load at the tile's end
        self.PFA, self.PFL = pfa, pfl
        self.PF = 0 if (dbuf or nomem) else pfa + pfl
        if self.PF:
            assert self.PF <= 2 * (self.NS * P // 4)
            self.vPF = self.nvgpr
            self.nvgpr += 1
        self.handlers = {}
        # real lane bits below this transpose with a slot through LDS
        # (gen_tr_lds), the others by DPP / v_permlane*_swap
        self.tr_lds = TR_LDS
        self.hstart = None       # first body line of the handler being generated
        self.swap_tmp = 0        # rotating temporary of swap_vals
        self.lane_ctrl = False   # generating a ctrl-2 (lane controls only) handler
        self.buf = None          # straight-line region being collected for scheduling
        # fp32 packed math: while set, value operands are 64-bit pairs holding
        # registers j and j + 1 and arithmetic is v_pk_*_f32 (pk_fix)
        self.packed = False

    # ---- helpers --------------------------------------------------------
    def e(self, s):
        if self.packed and s.startswith("v_pk_"):
            s = pk_fix(s)
        if self.buf is not None:
            self.buf.append(s)
        else:
            self.lines.append("\t" + s)

    def region(self):
        """Start collecting a straight-line VALU region (no DPP, no scalar
        ops, no branches) to be list-scheduled by end_region()."""
        self.buf = []

    def end_region(self):
        body, self.buf = self.buf, None
        for ins in schedule(body):
            self.lines.append("\t" + ins)

    def label(self, name):
        self.lines.append(name + ":")

    def re(self, j):
        return self.P * j

    def im(self, j):
        return self.P * (self.NS + j)

    def vp(self, r):
        return f"v[{r}:{r + 1}]" if (self.P == 2 or self.packed) else f"v{r}"

    def bc(self, r):  # a per-lane value used by every register: broadcast in packed math
        return f"B{r}" if self.packed else self.vp(r)

    def sm(self, k):  # coefficient m[k] in SGPRs (f64 m[8] / f32 m[16] of the op record)
        if self.packed:
            return f"S{k}"   # broadcast of s(76 + k), resolved by pk_fix
        return f"s[{76 + 2 * k}:{77 + 2 * k}]" if self.P == 2 else f"s{76 + k}"

    def op(self, name):  # "fma" -> "v_fma_f64" / "v_fma_f32" (packed: "v_pk_fma_f32")
        if self.packed:
            return f"v_pk_{name}_f32"
        return f"v_{name}_{self.F}"

    def mov(self):
        return "v_mov_b64" if self.packed else self.MOV

    def tmps(self, n, ts):
        """n temporaries of set ts: packed math takes even-aligned pairs."""
        if self.packed:
            return [self.D + 2 * ((ts * n + k) % (self.NT // 2)) for k in range(n)]
        return [self.T[(n * ts + k) % 16] for k in range(n)]

    def negate(self, r):
        """Flip the sign of the value at r (packed: of registers r and r + 1)."""
        if self.packed:
            self.e(f"v_pk_add_f32 v[{r}:{r + 1}], -v[{r}:{r + 1}], 0")
        else:
            self.e(f"v_xor_b32_e32 v{self.hi(r)}, 0x80000000, v{self.hi(r)}")

    def pk_regs(self, js):
        """Packed math applies to registers j, j + 1 at once: the even j of
        js when every such pair is in js (else None: scalar code)."""
        if not (PK and self.P == 1):
            return None
        st = set(js)
        ev = [j for j in js if j % 2 == 0]
        if len(ev) * 2 != len(js) or any(j + 1 not in st for j in ev):
            return None
        return ev

    def hi(self, r):     # dword holding the sign bit of the value at r
        return r + self.P - 1

    def handler(self, idx, name):
        self.finish_handler()
        lab = f"wh_{name}"
        self.handlers[idx] = lab
        self.lines.append("")
        self.lines.append(f"\t.p2align 2")
        self.label(lab)
        self.hstart = len(self.lines)

    def finish_handler(self):
        """Prologue of the handler just generated: copy the fields of its op
        record that its body reads (s68..s91) out of the prefetch buffer
        s[36:59], then prefetch the next record into the buffer.  A handler
        copies only what it uses (a CNOT its two control words, a rotation
        two coefficients) instead of every handler copying all 24 dwords."""
        if self.hstart is None:
            return
        used = set()
        for ln in self.lines[self.hstart:]:
            for a, b in re.findall(r"s\[(\d+):(\d+)\]", ln):
                used.update(range(int(a), int(b) + 1))
            for a in re.findall(r"\bs(\d+)\b", ln):
                used.add(int(a))
        used = sorted(d for d in used if REC_LO <= d <= REC_HI)
        # record bytes 64-95 (s84..s91: fp64 m[4..7], read by general 2x2s and
        # channels) are not prefetched: a handler that reads them loads them
        # from its own record here, beside the next record's prefetch
        hi = [d for d in used if d >= REC_HI - 7]
        used = [d for d in used if d < REC_HI - 7]
        pro = [f"\ts_load_dwordx8 s[{REC_HI - 7}:{REC_HI}], s[94:95], 0x40"] if hi else []
        k = 0
        while k < len(used):
            d = used[k]
            if d % 2 == 0 and k + 1 < len(used) and used[k + 1] == d + 1:
                pro.append(f"\ts_mov_b64 s[{d}:{d + 1}], s[{d - 32}:{d - 31}]")
                k += 2
            else:
                pro.append(f"\ts_mov_b32 s{d}, s{d - 32}")
                k += 1
        # (the host keeps the op records inside one 4 GiB-aligned window: no
        # carry into s95)
        pro += ["\ts_add_u32 s94, s94, 96",
                "\ts_load_dwordx16 s[36:51], s[94:95], 0x0"]
        if hi:
            pro.append("\ts_waitcnt lgkmcnt(0)")
        self.lines[self.hstart:self.hstart] = pro
        self.hstart = None

    def back(self):
        self.next_op()

    def next_op(self):
        """Start the next op (inlined at the end of every handler: one taken
        branch per op).  Op k+1's record was prefetched into s[36:59] by op
        k's prologue; op k+1's own prologue copies the fields it reads to
        s[68:91] and prefetches op k+2 (finish_handler).  The list ends with a
        sentinel record whose handler is the store epilogue; ops that need
        tile / wave predicates have bit 31 of the handler offset set and take
        the shared check path (rare)."""
        e = self.e
        e("s_waitcnt lgkmcnt(0)")
        # (ops with tile / wave predicates name the shared check path as their
        # handler; their own handler rides in the record's cWave word)
        e("s_add_u32 s18, s92, s36")                   # kernel base + handler offset (no carry: host-checked)
        e("s_setpc_b64 s[18:19]")

    def check_path(self):
        """Shared slow path (handler table entry "check"): an op with tile or
        wave predicates names it as its handler.  Skip the op (prefetch the one
        after it and start that) unless the tile satisfies its out-of-tile
        controls and this wave its wave-bit controls, else jump to the op's own
        handler, bits 8.. of the cWave word (s42; bits 0-7 the wave bits).
        The record is still in the prefetch buffer s[36:59]."""
        e = self.e
        self.label("wh_CHECK")
        self.handlers[LAYOUT["check"]] = "wh_CHECK"
        e("s_and_b64 s[96:97], s[32:33], s[40:41]")    # ctrlOut of the op
        e("s_cmp_eq_u64 s[96:97], s[40:41]")
        e("s_cbranch_scc0 .Lskip_op")
        # cWaveZero bit 31: out-of-tile bits that must be 0 in record bytes
        # 48-55 (a DIAG's spare m[2]; folded diagonal runs)
        e("s_bitcmp1_b32 s43, 31")
        e("s_cbranch_scc0 .Lcheck_zero_done")
        e("s_and_b64 s[96:97], s[32:33], s[48:49]")
        e("s_cmp_eq_u64 s[96:97], 0")
        e("s_cbranch_scc0 .Lskip_op")
        self.label(".Lcheck_zero_done")
        if self.W:
            e("s_and_b32 s97, s42, 0xff")
            e("s_and_b32 s96, s3, s97")                 # wave bits that must be 1
            e("s_cmp_eq_u32 s96, s97")
            e("s_cbranch_scc0 .Lskip_op")
            e("s_and_b32 s96, s3, s43")                 # wave bits that must be 0
            e("s_cmp_eq_u32 s96, 0")
            e("s_cbranch_scc0 .Lskip_op")
        e("s_lshr_b32 s18, s42, 8")
        e("s_add_u32 s18, s92, s18")
        e("s_setpc_b64 s[18:19]")
        self.label(".Lskip_op")
        e("s_add_u32 s94, s94, 96")
        e("s_load_dwordx16 s[36:51], s[94:95], 0x0")   # (record bytes 0-63; see finish_handler)
        e("s_branch .Lnext")

    # ---- predication: exec = lanes whose controls hold; registers j whose
    # slot controls fail are branched over (the record's cReg word carries
    # the host-computed mask of the registers that pass, bit j) ----
    def ctrl_begin(self):
        # LM (s[96:97]) = lanes with (lane & cLane) == cLane
        self.e(f"v_xor_b32_e32 v{self.vTmp}, s71, v{self.vLane}")   # aux: lane bits the planner flipped
        self.e(f"v_and_b32_e32 v{self.vTmp}, s70, v{self.vTmp}")
        self.e(f"v_cmp_eq_u32_e64 s[96:97], s70, v{self.vTmp}")
        if not NOP_FREE_EXEC:
            self.e("s_nop 4")
        self.e("s_mov_b64 exec, s[96:97]")   # (an SALU read of a VALU-written SGPR is interlocked)

    def ctrl_j(self, j, skip):
        self.e(f"s_bitcmp1_b32 s69, {j}")
        self.e(f"s_cbranch_scc0 {skip}")

    def ctrl_end(self):
        self.e("s_mov_b64 exec, -1")

    # ---- pair math (in place, registers of j and f) ---------------------
    def pair(self, kind, j, f, ts=0):
        r0, i0, r1, i1 = self.vp(self.re(j)), self.vp(self.im(j)), self.vp(self.re(f)), self.vp(self.im(f))
        T = [self.vp(t) for t in self.tmps(4, ts)]
        m = self.sm
        e = self.e
        # every kind updates the pair in place: products that still need the
        # old values go to temporaries first, the last op of each output is an
        # FMA into its own register (no copies back from temporaries)
        if kind == "M2":
            # T = m01 b, U = m10 a ; a = m00 a + T ; b = m11 b + U
            e(f"{self.op('mul')} {T[0]}, {m(2)}, {r1}")
            e(f"{self.op('mul')} {T[1]}, {m(2)}, {i1}")
            e(f"{self.op('mul')} {T[2]}, {m(4)}, {r0}")
            e(f"{self.op('mul')} {T[3]}, {m(4)}, {i0}")
            e(f"{self.op('fma')} {T[0]}, -{m(3)}, {i1}, {T[0]}")
            e(f"{self.op('fma')} {T[1]}, {m(3)}, {r1}, {T[1]}")
            e(f"{self.op('fma')} {T[2]}, -{m(5)}, {i0}, {T[2]}")
            e(f"{self.op('fma')} {T[3]}, {m(5)}, {r0}, {T[3]}")
            e(f"{self.op('fma')} {T[0]}, -{m(1)}, {i0}, {T[0]}")
            e(f"{self.op('fma')} {T[1]}, {m(1)}, {r0}, {T[1]}")
            e(f"{self.op('fma')} {T[2]}, -{m(7)}, {i1}, {T[2]}")
            e(f"{self.op('fma')} {T[3]}, {m(7)}, {r1}, {T[3]}")
            e(f"{self.op('fma')} {r0}, {m(0)}, {r0}, {T[0]}")
            e(f"{self.op('fma')} {i0}, {m(0)}, {i0}, {T[1]}")
            e(f"{self.op('fma')} {r1}, {m(6)}, {r1}, {T[2]}")
            e(f"{self.op('fma')} {i1}, {m(6)}, {i1}, {T[3]}")
        elif kind == "M2R":   # m = m00 m01 m10 m11 (real)
            e(f"{self.op('mul')} {T[0]}, {m(1)}, {r1}")
            e(f"{self.op('mul')} {T[1]}, {m(2)}, {r0}")
            e(f"{self.op('mul')} {T[2]}, {m(1)}, {i1}")
            e(f"{self.op('mul')} {T[3]}, {m(2)}, {i0}")
            e(f"{self.op('fma')} {r0}, {m(0)}, {r0}, {T[0]}")
            e(f"{self.op('fma')} {r1}, {m(3)}, {r1}, {T[1]}")
            e(f"{self.op('fma')} {i0}, {m(0)}, {i0}, {T[2]}")
            e(f"{self.op('fma')} {i1}, {m(3)}, {i1}, {T[3]}")
        elif kind == "M2RI":  # m = m00, Im m01, Im m10, m11
            # r0 = m0 r0 - m1 i1 ; i0 = m0 i0 + m1 r1 ; r1 = m3 r1 - m2 i0 ; i1 = m3 i1 + m2 r0
            e(f"{self.op('mul')} {T[0]}, -{m(1)}, {i1}")
            e(f"{self.op('mul')} {T[1]}, {m(1)}, {r1}")
            e(f"{self.op('mul')} {T[2]}, -{m(2)}, {i0}")
            e(f"{self.op('mul')} {T[3]}, {m(2)}, {r0}")
            e(f"{self.op('fma')} {r0}, {m(0)}, {r0}, {T[0]}")
            e(f"{self.op('fma')} {i0}, {m(0)}, {i0}, {T[1]}")
            e(f"{self.op('fma')} {r1}, {m(3)}, {r1}, {T[2]}")
            e(f"{self.op('fma')} {i1}, {m(3)}, {i1}, {T[3]}")
        elif kind == "ANTI":  # m = m01 re,im ; m10 re,im
            e(f"{self.op('mul')} {T[0]}, {m(0)}, {r1}")
            e(f"{self.op('fma')} {T[0]}, -{m(1)}, {i1}, {T[0]}")
            e(f"{self.op('mul')} {T[1]}, {m(0)}, {i1}")
            e(f"{self.op('fma')} {T[1]}, {m(1)}, {r1}, {T[1]}")
            e(f"{self.op('mul')} {r1}, {m(2)}, {r0}")
            e(f"{self.op('fma')} {r1}, -{m(3)}, {i0}, {r1}")
            e(f"{self.op('mul')} {i1}, {m(2)}, {i0}")
            e(f"{self.op('fma')} {i1}, {m(3)}, {r0}, {i1}")
            e(f"{self.mov()} {r0}, {T[0]}")
            e(f"{self.mov()} {i0}, {T[1]}")
        elif kind == "SWAP":
            for a, b in ((self.re(j), self.re(f)), (self.im(j), self.im(f))):
                self.swap_vals(a, b)
        elif kind == "ROTY":   # (a, b) -> (c a - s b, s a + c b) on re and im: m = tan(phi/2), sin(phi)
            for base in (self.re, self.im):
                self.rot(base(j), base(f), False)
        elif kind == "ROTX":   # a -> c a - i s b, b -> -i s a + c b: (a_im, b_re) by +phi, (a_re, b_im) by -phi
            self.rot(self.im(j), self.re(f), False)
            self.rot(self.re(j), self.im(f), True)
        elif kind == "HADD":   # (a, b) -> (a + b, a - b), unnormalised
            for base in (self.re, self.im):
                a, b = self.vp(base(j)), self.vp(base(f))
                e(f"{self.op('add')} {b}, {a}, -{b}")
                e(f"{self.op('fma')} {a}, 2.0, {a}, -{b}")
        elif kind in ("YSW", "YSWC"):
            # Y: a -> -i b, b -> i a  (YSWC: -Y): swap a_re <-> b_im, a_im <-> b_re, then two sign flips
            for x, y in ((self.re(j), self.im(f)), (self.im(j), self.re(f))):
                self.swap_vals(x, y)
            neg = (self.im(j), self.re(f)) if kind == "YSW" else (self.re(j), self.im(f))
            for r in neg:
                self.negate(r)
        else:
            raise ValueError(kind)

    def swap_vals(self, a, b):
        """Exchange the values at registers a and b.  fp64: three v_mov_b64
        through a temporary (rotating over the temporaries) -- on gfx950 the
        bench ran 4.5 % faster than with two v_swap_b32 per value
        (WAVE_SWAP64=0 keeps the swaps)."""
        e = self.e
        if self.packed:   # two fp32 values: 64-bit moves through a temporary pair
            t = self.D + 2 * (self.swap_tmp % (self.NT // 2))
            self.swap_tmp += 1
            e(f"v_mov_b64 v[{t}:{t + 1}], v[{a}:{a + 1}]")
            e(f"v_mov_b64 v[{a}:{a + 1}], v[{b}:{b + 1}]")
            e(f"v_mov_b64 v[{b}:{b + 1}], v[{t}:{t + 1}]")
            return
        if SWAP64 and self.P == 2:
            t = self.T[self.swap_tmp % self.NT]
            self.swap_tmp += 1
            e(f"v_mov_b64 v[{t}:{t + 1}], v[{a}:{a + 1}]")
            e(f"v_mov_b64 v[{a}:{a + 1}], v[{b}:{b + 1}]")
            e(f"v_mov_b64 v[{b}:{b + 1}], v[{t}:{t + 1}]")
            return
        for d in range(self.P):
            e(f"v_swap_b32 v{a + d}, v{b + d}")

    def rot(self, x, y, neg):
        """Rotate the register pair (x, y) by phi (neg: by -phi) in place with
        three shears: x -= t y; y += s x; x -= t y  (t = tan(phi/2) in m[0],
        s = sin(phi) in m[1]): 3 FMAs per pair instead of 4 multiplies + adds."""
        t, sn = self.sm(0), self.sm(1)
        mt, ps = (t, "-" + sn) if neg else ("-" + t, sn)
        X, Y = self.vp(x), self.vp(y)
        self.e(f"{self.op('fma')} {X}, {mt}, {Y}, {X}")
        self.e(f"{self.op('fma')} {Y}, {ps}, {X}, {Y}")
        self.e(f"{self.op('fma')} {X}, {mt}, {Y}, {X}")

    def cmul_sgpr(self, j, kr, ki, ts=0):
        # (x + iy) *= (m[kr] + i m[ki])
        x, y = self.vp(self.re(j)), self.vp(self.im(j))
        T = [self.vp(t) for t in self.tmps(2, ts)]
        self.e(f"{self.op('mul')} {T[0]}, {self.sm(ki)}, {y}")
        self.e(f"{self.op('mul')} {T[1]}, {self.sm(ki)}, {x}")
        self.e(f"{self.op('fma')} {x}, {self.sm(kr)}, {x}, -{T[0]}")
        self.e(f"{self.op('fma')} {y}, {self.sm(kr)}, {y}, {T[1]}")

    def cmul_vgpr(self, j, cr, ci, ts=0):
        x, y = self.vp(self.re(j)), self.vp(self.im(j))
        T = [self.vp(t) for t in self.tmps(2, ts)]
        self.e(f"{self.op('mul')} {T[0]}, {self.bc(ci)}, {y}")
        self.e(f"{self.op('mul')} {T[1]}, {self.bc(ci)}, {x}")
        self.e(f"{self.op('fma')} {x}, {self.bc(cr)}, {x}, -{T[0]}")
        self.e(f"{self.op('fma')} {y}, {self.bc(cr)}, {y}, {T[1]}")

    # ---- handlers --------------------------------------------------------
    def lane_exec_begin(self):
        """ctrl 2 (controls on lane bits only): exec = the lanes whose cLane
        bits are set, no per-register tests."""
        self.ctrl_begin()

    def gen_slot(self, kind, s, ctrl):
        self.handler(idx_slot(kind, s, ctrl), f"{kind}_s{s}_c{ctrl}")
        if ctrl == 2:
            self.lane_exec_begin()
            ctrl = 0
            self.lane_ctrl = True
        if ctrl:
            self.ctrl_begin()
        else:
            self.region()
        js = [j for j in range(self.NS) if not (j >> s) & 1]
        ev = self.pk_regs(js) if (not ctrl and kind != "SWAP") else None
        if self.P == 1 and kind == "SWAP" and not ctrl and SWAP64:
            self.swap_pairs32(s)
        elif ev:
            self.packed = True
            for p, j in enumerate(ev):
                self.pair(kind, j, j | (1 << s), p % 4)
            self.packed = False
        else:
            for p, j in enumerate(js):
                f = j | (1 << s)
                if ctrl:
                    skip = f".Lskip_{kind}_{s}_{j}"
                    self.ctrl_j(j, skip)
                    self.pair(kind, j, f)
                    self.label(skip)
                else:
                    self.pair(kind, j, f, p % 4)
        if ctrl:
            self.ctrl_end()
        else:
            self.end_region()
        self.lane_ctrl_end()
        self.back()

    def gen_swk(self, lane, t, c, v):
        """X on slot t (lane = 0) or on lane bit t (lane = 1) of the registers
        j whose slot-c bit is v: a CNOT whose control sits in a slot.  The
        generic controlled handler tests every register's bit of the record's
        mask (32 scalar tests, up to 16 taken branches, its moves unscheduled);
        here the registers are fixed, the moves list-scheduled.  Lane controls
        still set exec (ctrl_begin)."""
        self.handler(idx_swk(lane, t, c, v), f"SWK_{'l' if lane else 's'}{t}_c{c}_v{v}")
        e = self.e
        if lane:
            e("s_nop 1")
        self.ctrl_begin()
        if lane:
            for j in range(self.NS):
                if ((j >> c) & 1) != v:
                    continue
                for r in [self.re(j) + d for d in range(self.P)] + [self.im(j) + d for d in range(self.P)]:
                    e(f"ds_swizzle_b32 v{r}, v{r} offset:{0x1f | ((1 << t) << 10):#x}")
        else:
            self.region()
            for j in range(self.NS):
                if not (j >> t) & 1 and ((j >> c) & 1) == v:
                    self.pair("SWAP", j, j | (1 << t))
            self.end_region()
        self.ctrl_end()
        self.back()

    def swap_pairs32(self, s):
        """fp32 X on slot s, every register pair: adjacent values move as 64-bit
        pairs (s >= 1: registers j, j+1 with j and j + 2^s; s = 0: the two
        halves of one 64-bit register, one v_pk_mov_b32)."""
        e = self.e
        for base in (self.re, self.im):
            if s == 0:
                for j in range(0, self.NS, 2):
                    r = base(j)
                    e(f"v_pk_mov_b32 v[{r}:{r + 1}], v[{r}:{r + 1}], v[{r}:{r + 1}] op_sel:[1,0]")
                continue
            for j in range(0, self.NS, 2):
                if (j >> s) & 1:
                    continue
                a, b = base(j), base(j | (1 << s))
                t = self.T[self.swap_tmp % (self.NT // 2) * 2]   # two adjacent fp32 temporaries
                self.swap_tmp += 1
                e(f"v_mov_b64 v[{t}:{t + 1}], v[{a}:{a + 1}]")
                e(f"v_mov_b64 v[{a}:{a + 1}], v[{b}:{b + 1}]")
                e(f"v_mov_b64 v[{b}:{b + 1}], v[{t}:{t + 1}]")

    def lane_ctrl_end(self):
        if self.lane_ctrl:
            self.ctrl_end()
            self.lane_ctrl = False

    def gen_slot2(self, kind, s, ctrl):
        self.handler(idx_slot2(kind, s, ctrl), f"{kind}_s{s}_c{ctrl}")
        if ctrl == 2:
            self.lane_exec_begin()
            ctrl = 0
            self.lane_ctrl = True
        if ctrl:
            self.ctrl_begin()
        else:
            self.region()
        js = [j for j in range(self.NS) if not (j >> s) & 1]
        ev = None if ctrl else self.pk_regs(js)
        if ev:
            self.packed = True
            for p, j in enumerate(ev):
                self.pair(kind, j, j | (1 << s), p % 4)
            self.packed = False
            js = []
        for p, j in enumerate(js):
            f = j | (1 << s)
            if ctrl:
                skip = f".Lskip_{kind}_{s}_{j}"
                self.ctrl_j(j, skip)
                self.pair(kind, j, f)
                self.label(skip)
            else:
                self.pair(kind, j, f)
        if ctrl:
            self.ctrl_end()
        else:
            self.end_region()
        self.lane_ctrl_end()
        self.back()

    def gen_ph(self, kind, creg, lane):
        """Unit-modulus phase (DSC: a real factor) on the registers j with
        (j & creg) == creg of the lanes whose cLane (s70) bits are set (lane =
        1; exec-masked)."""
        self.handler(idx_ph(kind, creg, lane), f"{kind}_m{creg}_l{lane}")
        e = self.e
        if lane:
            e(f"v_xor_b32_e32 v{self.vTmp}, s71, v{self.vLane}")
            e(f"v_and_b32_e32 v{self.vTmp}, s70, v{self.vTmp}")
            e(f"v_cmp_eq_u32_e64 s[96:97], s70, v{self.vTmp}")
            if not NOP_FREE_EXEC:
                e("s_nop 4")
            e("s_mov_b64 exec, s[96:97]")
        self.region()
        js = [j for j in range(self.NS) if (j & creg) == creg]
        ev = self.pk_regs(js)
        if ev:
            self.packed = True
            js = ev
        for j in js:
            x, y = self.re(j), self.im(j)
            if kind in ("DNEG", "DROTN"):
                self.negate(x)
                self.negate(y)
            if kind in ("DROT", "DROTN"):
                self.rot(x, y, False)
            elif kind in ("DMULI", "DMULNI"):   # x + iy -> -y + ix  /  y - ix
                self.swap_vals(x, y)
                self.negate(x if kind == "DMULI" else y)
            elif kind == "DSC":   # real factor: two multiplies instead of a complex product
                e(f"{self.op('mul')} {self.vp(x)}, {self.sm(0)}, {self.vp(x)}")
                e(f"{self.op('mul')} {self.vp(y)}, {self.sm(0)}, {self.vp(y)}")
        self.packed = False
        self.end_region()
        if lane:
            e("s_mov_b64 exec, -1")
        self.back()

    def gen_ch(self, kind, a, b):
        self.handler(idx_ch(kind, a, b), f"{kind}_a{a}_b{b}")
        e = self.e
        self.region()
        k = 0
        js = [j for j in range(self.NS) if not ((j >> a) & 1 or (j >> b) & 1)]
        ev = self.pk_regs(js)
        if ev:
            self.packed = True
            js = ev
        for j in js:
            x = [j, j | (1 << a), j | (1 << b), j | (1 << a) | (1 << b)]
            for base in (self.re, self.im):
                X = [self.vp(base(r)) for r in x]
                e(f"{self.op('mul')} {X[1]}, {self.sm(4)}, {X[1]}")
                e(f"{self.op('mul')} {X[2]}, {self.sm(4)}, {X[2]}")
                if kind == "CH1":
                    T = self.vp(self.tmps(1, k)[0])
                    k += 1
                    e(f"{self.op('mul')} {T}, {self.sm(2)}, {X[0]}")
                    e(f"{self.op('mul')} {X[0]}, {self.sm(0)}, {X[0]}")
                    e(f"{self.op('fma')} {X[0]}, {self.sm(1)}, {X[3]}, {X[0]}")
                    e(f"{self.op('fma')} {X[3]}, {self.sm(3)}, {X[3]}, {T}")
        self.packed = False
        self.end_region()
        self.back()

    def gen_d2s(self, s, ctrl):
        self.handler(idx_d2s(s, ctrl), f"D2S_s{s}_c{ctrl}")
        if ctrl == 2:
            self.lane_exec_begin()
            ctrl = 0
            self.lane_ctrl = True
        if ctrl:
            self.ctrl_begin()
        else:
            self.region()
        js = list(range(self.NS))
        ev = self.pk_regs(js) if (not ctrl and s >= 1) else None
        if ev:   # registers j, j + 1 share slot bit s >= 1: the same coefficients
            self.packed = True
            for j in ev:
                one = (j >> s) & 1
                self.cmul_sgpr(j, 2 if one else 0, 3 if one else 1, j % 8)
            self.packed = False
            js = []
        for j in js:
            one = (j >> s) & 1
            if ctrl:
                skip = f".Lskip_d2s_{s}_{j}"
                self.ctrl_j(j, skip)
                self.cmul_sgpr(j, 2 if one else 0, 3 if one else 1)
                self.label(skip)
            else:
                self.cmul_sgpr(j, 2 if one else 0, 3 if one else 1, j % 8)
        if ctrl:
            self.ctrl_end()
        else:
            self.end_region()
        self.lane_ctrl_end()
        self.back()

    def gen_d2l(self, ctrl):
        self.handler(idx_d2l(ctrl), f"D2L_c{ctrl}")
        # per-lane coefficient: lane bit m[4] (its low dword) ? d1 : d0
        self.e(f"v_bfe_u32 v{self.vTmp}, v{self.vLane}, s{76 + 4 * self.P}, 1")
        self.e(f"v_cmp_ne_u32_e64 {SEL}, 0, v{self.vTmp}")
        C0, C1, T0, T1 = self.C0, self.C1, self.T[14], self.T[15]
        self.e(f"{self.MOV} {self.vp(C0)}, {self.sm(0)}")
        self.e(f"{self.MOV} {self.vp(C1)}, {self.sm(1)}")
        self.e(f"{self.MOV} {self.vp(T0)}, {self.sm(2)}")
        self.e(f"{self.MOV} {self.vp(T1)}, {self.sm(3)}")
        for c, t in ((C0, T0), (C1, T1)):
            for d in range(self.P):
                self.e(f"v_cndmask_b32_e64 v{c + d}, v{c + d}, v{t + d}, {SEL}")
        if ctrl:
            self.ctrl_begin()
        else:
            self.region()
        js = list(range(self.NS))
        ev = None if ctrl else self.pk_regs(js)
        if ev:
            self.packed = True
            for j in ev:
                self.cmul_vgpr(j, C0, C1, j % 7)
            self.packed = False
            js = []
        for j in js:
            if ctrl:
                skip = f".Lskip_d2l_{j}"
                self.ctrl_j(j, skip)
                self.cmul_vgpr(j, C0, C1)
                self.label(skip)
            else:
                self.cmul_vgpr(j, C0, C1, j % 7)
        if ctrl:
            self.ctrl_end()
        else:
            self.end_region()
        self.back()

    def gen_diag(self, creg, lane):
        """Phase m[0] + i m[1] on the registers j with (j & creg) == creg
        (chosen here, at generation time) of the lanes whose cLane bits are 1
        (lane = 1: per-lane phase, 1 on the other lanes)."""
        self.handler(idx_diag(creg, lane), f"DIAG_m{creg}_l{lane}")
        e = self.e
        js = [j for j in range(self.NS) if (j & creg) == creg]
        ev = self.pk_regs(js)
        if not lane:
            self.region()
            self.packed = bool(ev)
            for k, j in enumerate(ev or js):
                self.cmul_sgpr(j, 0, 1, k % 8)
            self.packed = False
            self.end_region()
            self.back()
            return
        C0, C1 = self.C0, self.C1
        e(f"v_xor_b32_e32 v{self.vTmp}, s71, v{self.vLane}")
        e(f"v_and_b32_e32 v{self.vTmp}, s70, v{self.vTmp}")
        e(f"v_cmp_eq_u32_e64 {SEL}, s70, v{self.vTmp}")
        e(f"{self.MOV} {self.vp(C0)}, {self.sm(0)}")
        e(f"{self.MOV} {self.vp(C1)}, {self.sm(1)}")
        if self.P == 2:
            e(f"v_cndmask_b32_e64 v{C0}, 0, v{C0}, {SEL}")
            e(f"v_mov_b32_e32 v{self.vTmp}, 0x3ff00000")   # hi dword of 1.0 (a literal cannot ride in VOP3)
            e(f"v_cndmask_b32_e64 v{C0 + 1}, v{self.vTmp}, v{C0 + 1}, {SEL}")
            e(f"v_cndmask_b32_e64 v{C1}, 0, v{C1}, {SEL}")
            e(f"v_cndmask_b32_e64 v{C1 + 1}, 0, v{C1 + 1}, {SEL}")
        else:
            e(f"v_cndmask_b32_e64 v{C0}, 1.0, v{C0}, {SEL}")
            e(f"v_cndmask_b32_e64 v{C1}, 0, v{C1}, {SEL}")
        self.region()
        self.packed = bool(ev)
        for k, j in enumerate(ev or js):
            self.cmul_vgpr(j, C0, C1, k % 8)
        self.packed = False
        self.end_region()
        self.back()

    def gen_tr_lds(self, s, l):
        """Transpose slot s with real lane bit l through this wave's LDS
        outbox (no other wave reads it: no barrier).  A lane with bit l clear
        gives its registers with slot bit s set and takes the partner's with
        it clear, a lane with the bit set the other way round: each lane
        writes the half it gives to its own 64-byte slot (exec = the lanes of
        one kind at a time), then reads the partner's slot into the same
        registers -- two rounds (re, im) of 64 bytes per lane.  A handful of
        VALU instructions instead of 80-128 DPP moves and selects."""
        e = self.e
        vt, vl = self.vTmp, self.vLane
        e("s_nop 1")   # VALU write -> LDS read of the same VGPR
        # chunk k of lane L at k * 1 KiB + 16 L: the 64 lanes of one
        # ds_*_b128 cover 1 KiB contiguously (no bank conflicts)
        e(f"s_mul_i32 s97, s3, {self.OUTBOX}")
        e(f"v_lshlrev_b32_e32 v{vt}, 4, v{vl}")
        e(f"v_add_u32_e32 v{vt}, s97, v{vt}")
        clear = 0
        for lane in range(64):
            if not (lane >> l) & 1:
                clear |= 1 << lane
        e(f"s_mov_b32 s96, {clear & 0xffffffff:#x}")
        e(f"s_mov_b32 s97, {clear >> 32:#x}")
        js = [j for j in range(self.NS) if not (j >> s) & 1]
        per = 4 // self.P                    # values per 16-byte LDS move
        for base in (self.re, self.im):
            # register blocks: consecutive j (bit s clear) with their f = j | 2^s
            blocks = []
            for k in range(0, len(js), per):
                grp = js[k:k + per]
                assert grp == list(range(grp[0], grp[0] + per)), "TR via LDS: registers not adjacent"
                blocks.append((base(grp[0]), base(grp[0] | (1 << s))))
            assert len(blocks) * 16 <= 64
            for phase in ("w", "r"):
                if phase == "r":
                    e("s_waitcnt lgkmcnt(0)")
                    e(f"v_xor_b32_e32 v{vt}, {16 << l}, v{vt}")     # the partner's slot
                for kind in ("clear", "set"):
                    e("s_mov_b64 exec, s[96:97]" if kind == "clear" else "s_not_b64 exec, s[96:97]")
                    for k, (jr, fr) in enumerate(blocks):
                        r = fr if kind == "clear" else jr
                        if phase == "w":
                            e(f"ds_write_b128 v{vt}, v[{r}:{r + 3}] offset:{1024 * k}")
                        else:
                            e(f"ds_read_b128 v[{r}:{r + 3}], v{vt} offset:{1024 * k}")
                e("s_mov_b64 exec, -1")
                if phase == "r":
                    e(f"v_xor_b32_e32 v{vt}, {16 << l}, v{vt}")     # back to ours
            e("s_waitcnt lgkmcnt(0)")
        self.back()

    def gen_tr(self, s, l):
        self.handler(idx_tr(s, l), f"TR_s{s}_l{l}")
        # (16-byte LDS moves need 16 bytes of adjacent registers with slot
        # bit s clear: s >= the vector bits, the only slots the planner moves)
        if l < self.tr_lds and s >= self.VB:
            self.gen_tr_lds(s, l)
            return
        e = self.e
        e("s_nop 1")  # VALU write -> DPP / permlane read of the same VGPR
        pairs = []
        for j in range(self.NS):
            if (j >> s) & 1:
                continue
            f = j | (1 << s)
            for base in (self.re, self.im):
                for d in range(self.P):
                    pairs.append((base(j) + d, base(f) + d))
        tmp = [self.D + i for i in range(min(8, self.NT * self.P))]   # the first dwords of the temporaries
        if l >= 4:
            op = "v_permlane32_swap_b32_e32" if l == 5 else "v_permlane16_swap_b32_e32"
            for a, b in pairs:
                e(f"{op} v{a}, v{b}")
            self.back()
            return
        if l >= 2:
            sh = 8 if l == 3 else 4
            lo_banks = "0x3" if l == 3 else "0x5"   # lanes with the bit clear
            hi_banks = "0xc" if l == 3 else "0xa"   # lanes with the bit set
            # all copies first (32 temporaries), then the DPP moves: one
            # VALU-write -> DPP-read wait for the whole handler
            G = self.NT * self.P               # dwords of temporaries
            big = [self.D + i for i in range(G)]
            for g in range(0, len(pairs), G):
                grp = pairs[g:g + G]
                for k, (a, b) in enumerate(grp):
                    if self.P == 2 and SWAP64:
                        # a value's two dwords are adjacent pairs: one 64-bit copy
                        if k % 2 == 0:
                            e(f"v_mov_b64 v[{big[k]}:{big[k] + 1}], v[{b}:{b + 1}]")
                    else:
                        e(f"v_mov_b32_e32 v{big[k]}, v{b}")
                e("s_nop 1")
                for k, (a, b) in enumerate(grp):
                    # bit clear: b <- partner(lane + sh).a ; bit set: a <- partner(lane - sh).b (old)
                    e(f"v_mov_b32_dpp v{b}, v{a} row_shl:{sh} row_mask:0xf bank_mask:{lo_banks}")
                    e(f"v_mov_b32_dpp v{a}, v{big[k]} row_shr:{sh} row_mask:0xf bank_mask:{hi_banks}")
            self.back()
            return
        qp = "[1,0,3,2]" if l == 0 else "[2,3,0,1]"
        e(f"v_and_b32_e32 v{self.vTmp}, {1 << l}, v{self.vLane}")
        e(f"v_cmp_ne_u32_e64 {SEL}, 0, v{self.vTmp}")
        per = len(tmp) // 2
        for g in range(0, len(pairs), per):
            grp = pairs[g:g + per]
            for k, (a, b) in enumerate(grp):
                e(f"v_mov_b32_dpp v{tmp[2 * k]}, v{b} quad_perm:{qp} row_mask:0xf bank_mask:0xf")
                e(f"v_mov_b32_dpp v{tmp[2 * k + 1]}, v{a} quad_perm:{qp} row_mask:0xf bank_mask:0xf")
            for k, (a, b) in enumerate(grp):
                # bit set: a <- partner's b ; bit clear: b <- partner's a
                e(f"v_cndmask_b32_e64 v{a}, v{a}, v{tmp[2 * k]}, {SEL}")
                e(f"v_cndmask_b32_e64 v{b}, v{tmp[2 * k + 1]}, v{b}, {SEL}")
            # the next group's DPPs read other registers: no hazard
        self.back()

    # ---- gates on lane bits 0-3 (no transposition) --------------------
    def lane_fetch(self, l, dst, src):
        """dst dword <- the partner lane's (lane ^ 2^l) src dword (WAVE_SWZ >= 3:
        through the LDS crossbar, the caller waits for lgkmcnt before use)."""
        if SWZ >= 3 and l <= 2:
            self.e(f"ds_swizzle_b32 v{dst}, v{src} offset:{0x1f | ((1 << l) << 10):#x}")
            return
        if l < 2:
            qp = "[1,0,3,2]" if l == 0 else "[2,3,0,1]"
            self.e(f"v_mov_b32_dpp v{dst}, v{src} quad_perm:{qp} row_mask:0xf bank_mask:0xf")
            return
        sh = 8 if l == 3 else 4
        lo, hi = ("0x3", "0xc") if l == 3 else ("0x5", "0xa")
        self.e(f"v_mov_b32_dpp v{dst}, v{src} row_shl:{sh} row_mask:0xf bank_mask:{lo}")
        self.e(f"v_mov_b32_dpp v{dst}, v{src} row_shr:{sh} row_mask:0xf bank_mask:{hi}")

    def lane_coeffs(self, kind, l):
        """Per-lane coefficients (SEL = lanes with bit l set): CS multiplies
        the lane's own amplitude, CP the partner's."""
        e = self.e
        e(f"v_bfe_u32 v{self.vTmp}, v{self.vLane}, {l}, 1")
        e(f"v_cmp_ne_u32_e64 {SEL}, 0, v{self.vTmp}")
        CL, C0 = self.CL, self.C0

        def sel(dst, k_clear, k_set):
            e(f"{self.MOV} {self.vp(dst)}, {self.sm(k_clear)}")
            if self.lean:
                # the coefficients live in C0 / C1: select dword by dword through vTmp
                for d in range(self.P):
                    e(f"v_mov_b32_e32 v{self.vTmp}, s{76 + self.P * k_set + d}")
                    e(f"v_cndmask_b32_e64 v{dst + d}, v{dst + d}, v{self.vTmp}, {SEL}")
                return
            e(f"{self.MOV} {self.vp(C0)}, {self.sm(k_set)}")
            for d in range(self.P):
                e(f"v_cndmask_b32_e64 v{dst + d}, v{dst + d}, v{C0 + d}, {SEL}")
        P = self.P
        if kind in ("M2R", "M2RI"):      # m00 m01 m10 m11 (M2RI: the off-diagonals imaginary)
            sel(CL, 0, 3)
            sel(CL + P, 1, 2)
        elif kind == "ANTI":             # m01 re,im ; m10 re,im
            sel(self.CLA, 0, 2)
            sel(self.CLA + P, 1, 3)
        elif kind == "M2":               # m00, m01, m10, m11 complex
            sel(CL, 0, 6)
            sel(CL + P, 1, 7)
            sel(CL + 2 * P, 2, 4)
            sel(CL + 3 * P, 3, 5)

    def lane_math(self, kind, j, px, py, B=None):
        x, y = self.vp(self.re(j)), self.vp(self.im(j))
        CS, CP = self.bc(self.CL), self.bc(self.CL + self.P)
        CSr, CSi, CPr, CPi = (self.bc(self.CL + self.P * k) for k in range(4))
        e = self.e
        px, py = self.vp(px), self.vp(py)
        if kind == "M2R":
            e(f"{self.op('mul')} {px}, {CP}, {px}")
            e(f"{self.op('mul')} {py}, {CP}, {py}")
            e(f"{self.op('fma')} {x}, {CS}, {x}, {px}")
            e(f"{self.op('fma')} {y}, {CS}, {y}, {py}")
        elif kind == "M2RI":
            e(f"{self.op('mul')} {py}, -{CP}, {py}")
            e(f"{self.op('mul')} {px}, {CP}, {px}")
            e(f"{self.op('fma')} {x}, {CS}, {x}, {py}")
            e(f"{self.op('fma')} {y}, {CS}, {y}, {px}")
        elif kind == "ANTI":
            CPr, CPi = self.bc(self.CLA), self.bc(self.CLA + self.P)
            e(f"{self.op('mul')} {x}, {CPr}, {px}")
            e(f"{self.op('mul')} {y}, {CPr}, {py}")
            e(f"{self.op('fma')} {x}, -{CPi}, {py}, {x}")
            e(f"{self.op('fma')} {y}, {CPi}, {px}, {y}")
        elif kind == "M2":
            B = self.vp(B)
            e(f"{self.op('mul')} {B}, {CPr}, {py}")
            e(f"{self.op('fma')} {B}, {CPi}, {px}, {B}")
            e(f"{self.op('mul')} {px}, {CPr}, {px}")
            e(f"{self.op('fma')} {px}, -{CPi}, {py}, {px}")
            e(f"{self.op('fma')} {px}, -{CSi}, {y}, {px}")
            e(f"{self.op('fma')} {B}, {CSi}, {x}, {B}")
            e(f"{self.op('fma')} {x}, {CSr}, {x}, {px}")
            e(f"{self.op('fma')} {y}, {CSr}, {y}, {B}")

    def gen_lane(self, kind, l, ctrl):
        """A one-qubit gate whose target is lane bit l: every lane combines
        its own amplitude with its partner's (lane ^ 2^l, fetched by DPP)
        using per-lane coefficients, in place -- instead of transposing the
        bit into a slot and back (2 x 64-128 VALU)."""
        self.handler(idx_lane(kind, l, ctrl), f"L{kind}_l{l}_c{ctrl}")
        e = self.e
        e("s_nop 1")   # VALU write -> DPP read of the same VGPR
        NS = self.NS
        if kind != "SWAP":
            self.lane_coeffs(kind, l)
        if ctrl:
            self.ctrl_begin()
        per = 3 if kind == "M2" else 2        # temporaries (doubles) per amplitude
        batch = 1 if ctrl else (2 if self.lean else (4 if kind == "M2" else 8))
        for j0 in range(0, NS, batch):
            js = list(range(j0, j0 + batch))
            skip = f".Lskip_L{kind}_{l}_{j0}"
            if ctrl:
                self.ctrl_j(j0, skip)
            if kind == "SWAP":
                for j in js:
                    regs = [self.re(j) + d for d in range(self.P)] + [self.im(j) + d for d in range(self.P)]
                    if (l == 2 and SWZ >= 1) or (l < 2 and SWZ >= 2):
                        # in place: every lane's dword is read at issue (the
                        # partner lane ^ 2^l is active whenever this one is:
                        # a lane control is never the target bit)
                        for r in regs:
                            e(f"ds_swizzle_b32 v{r}, v{r} offset:{0x1f | ((1 << l) << 10):#x}")
                    elif l < 2:
                        for r in regs:   # in place: DPP reads every lane before writing
                            self.lane_fetch(l, r, r)
                    else:
                        tmp = [self.D + k for k in range(2 * self.P)]
                        if self.P == 2:   # re and im as 64-bit copies
                            e(f"v_mov_b64 v[{tmp[0]}:{tmp[1]}], v[{regs[0]}:{regs[1]}]")
                            e(f"v_mov_b64 v[{tmp[2]}:{tmp[3]}], v[{regs[2]}:{regs[3]}]")
                        else:
                            for r, t in zip(regs, tmp):
                                e(f"v_mov_b32_e32 v{t}, v{r}")
                        e("s_nop 1")
                        for r, t in zip(regs, tmp):
                            self.lane_fetch(l, r, t)
            elif PK and self.P == 1 and not ctrl and kind != "M2" and batch == 2:
                # fp32: the two registers of the batch as one packed pair --
                # partners fetched into adjacent temporaries, one v_pk op per
                # two amplitudes (coefficients broadcast)
                j = js[0]
                px, py = self.D, self.D + 2
                for d, r in enumerate((self.re(j), self.re(j) + 1)):
                    self.lane_fetch(l, px + d, r)
                for d, r in enumerate((self.im(j), self.im(j) + 1)):
                    self.lane_fetch(l, py + d, r)
                if SWZ >= 3 and l <= 2:
                    e("s_waitcnt lgkmcnt(0)")
                self.region()
                self.packed = True
                self.lane_math(kind, j, px, py)
                self.packed = False
                self.end_region()
            else:
                slots = []
                for k, j in enumerate(js):
                    px, py = self.T[per * k], self.T[per * k + 1]
                    B = self.T[per * k + 2] if kind == "M2" else None
                    for d in range(self.P):
                        self.lane_fetch(l, px + d, self.re(j) + d)
                        self.lane_fetch(l, py + d, self.im(j) + d)
                    slots.append((j, px, py, B))
                if SWZ >= 3 and l <= 2:
                    e("s_waitcnt lgkmcnt(0)")
                if not ctrl:
                    self.region()
                for j, px, py, B in slots:
                    self.lane_math(kind, j, px, py, B)
                if not ctrl:
                    self.end_region()
            if ctrl:
                self.label(skip)
        if ctrl:
            self.ctrl_end()
        self.back()   # (next_op waits for lgkmcnt(0): the swizzles have landed)

    def gen_trw(self, s, b):
        """Transpose slot s with wave bit b through LDS: the wave with the bit
        clear sends its registers with slot bit s set and receives the
        partner's registers with it clear (and vice versa), in place."""
        self.handler(idx_trw(s, b), f"TRW_s{s}_b{b}")
        e = self.e
        vt, vl = self.vTmp, self.vLane
        # registers j .. j + chunk - 1 with the same slot bit s are adjacent
        # VGPRs: move them with one LDS instruction of up to 16 bytes
        chunk = min(1 << s, 4 // self.P)
        width = chunk * self.P            # dwords per LDS instruction
        lo_regs, hi_regs = [], []
        for j in range(0, self.NS, chunk):
            if (j >> s) & 1:
                continue
            f = j | (1 << s)
            lo_regs += [self.re(f), self.im(f)]
            hi_regs += [self.re(j), self.im(j)]
        ob = self.OUTBOX
        e(f"s_mul_i32 s96, s3, {ob}")
        e(f"v_lshlrev_b32_e32 v{vt}, {(4 * width).bit_length() - 1}, v{vl}")
        e(f"v_add_u32_e32 v{vt}, s96, v{vt}")
        # lean: the outbox holds half of the moved registers, two rounds
        rounds = 2 if self.lean else 1
        per = len(lo_regs) // rounds
        for rnd in range(rounds):
            for phase in ("w", "r"):
                tagp = f"{rnd}{phase}"
                e(f"s_bitcmp1_b32 s3, {b}")
                e(f"s_cbranch_scc1 .Ltrw_{s}_{b}_{tagp}hi")
                for regs, tag in ((lo_regs, "lo"), (hi_regs, "hi")):
                    if tag == "hi":
                        self.label(f".Ltrw_{s}_{b}_{tagp}hi")
                    for k, r in enumerate(regs[rnd * per:(rnd + 1) * per]):
                        stride = 64 * 4 * width
                        vr = f"v[{r}:{r + width - 1}]" if width > 1 else f"v{r}"
                        if phase == "w":
                            e(f"ds_write_b{32 * width} v{vt}, {vr} offset:{k * stride}")
                        else:
                            e(f"ds_read_b{32 * width} {vr}, v{vt} offset:{k * stride}")
                    if tag == "lo":
                        e(f"s_branch .Ltrw_{s}_{b}_{tagp}done")
                self.label(f".Ltrw_{s}_{b}_{tagp}done")
                if phase == "w" or rnd + 1 < rounds:
                    e(f"v_xor_b32_e32 v{vt}, {(1 << b) * ob}, v{vt}")   # the partner's outbox (and back)
                e("s_waitcnt lgkmcnt(0)")
                e("s_barrier")
        self.back()

    # ---- the kernel -------------------------------------------------------
    def kernel(self):
        R, NS, D = self.R, self.NS, self.D
        NG = NS * self.P // 4   # 16-byte groups per array per lane
        K = R + 6 + self.W  # tile bits
        L = self.lines
        L.append('\t.amdgcn_target "amdgcn-amd-amdhsa--gfx950"')
        L.append("\t.amdhsa_code_object_version 6")
        L.append("\t.text")
        L.append("\t.protected\tqa_wave_tile")
        L.append("\t.globl\tqa_wave_tile")
        L.append("\t.p2align\t8")
        L.append("\t.type\tqa_wave_tile,@function")
        self.label("qa_wave_tile")
        e = self.e
        vl, vldb, vstb, vt = self.vLane, self.vLdB, self.vStB, self.vTmp
        e("s_load_dwordx4 s[4:7], s[0:1], 0x0")       # re, im
        e("s_load_dwordx2 s[8:9], s[0:1], 0x10")      # launch record
        e("s_load_dword s100, s[0:1], 0x18")          # tile-index bits to insert (split launches)
        e(f"v_and_b32_e32 v{vl}, 63, v0")
        if self.W:
            # wave index in the workgroup (= its wave bits): lane 0's work-item id / 64
            e("v_readfirstlane_b32 s3, v0")
            e("s_nop 4")                          # VALU-written SGPR read by SALU / SMEM
            e("s_lshr_b32 s3, s3, 6")
            e(f"s_and_b32 s3, s3, {(1 << self.W) - 1}")
        else:
            e("s_mov_b32 s3, 0")
        e("s_getpc_b64 s[92:93]")
        self.label(".Lentry_pc")
        e("s_sub_u32 s92, s92, .Lentry_pc-qa_wave_tile")   # kernel base: handlers jump from here
        e("s_subb_u32 s93, s93, 0")
        e("s_waitcnt lgkmcnt(0)")
        # launch word bit 29: report the kernel base (vector stores of every
        # lane to debugBuf) and stop -- the host checks once that no handler
        # address carries into the high word, which next_op then never adds
        e("s_load_dword s52, s[8:9], 0x14")
        e("s_waitcnt lgkmcnt(0)")
        e("s_bitcmp1_b32 s52, 29")
        e("s_cbranch_scc0 .Lno_base_probe")
        e(f"s_load_dwordx2 s[52:53], s[8:9], {DEBUG_BUF}")
        e("s_waitcnt lgkmcnt(0)")
        e("v_mov_b32_e32 v128, s92")
        e("v_mov_b32_e32 v129, s93")
        e("v_mov_b32_e32 v130, 0")
        e("global_store_dwordx2 v130, v[128:129], s[52:53]")
        e("s_waitcnt vmcnt(0)")
        e("s_endpgm")
        self.label(".Lno_base_probe")
        e("s_mov_b32 s19, s93")                       # handler addresses: s[18:19] = {s92 + offset, s93}
        e("s_load_dwordx4 s[12:15], s[8:9], 0x0")     # numTiles, waveStride
        e("s_load_dwordx8 s[20:27], s[8:9], 0x18")    # pos[0..7]
        e("s_load_dwordx4 s[28:31], s[8:9], 0x38")    # pos[8..11]
        e(f"s_add_u32 s10, s8, {OPS_OFF}")
        e("s_addc_u32 s11, s9, 0")
        e(f"v_lshlrev_b32_e32 v{vt}, 2, v{vl}")
        e(f"global_load_dword v{vldb}, v{vt}, s[8:9] offset:344")
        e(f"global_load_dword v{vstb}, v{vt}, s[8:9] offset:600")
        # first tile = workgroup (one wave each)
        # first tile of this workgroup.  The dispatcher deals workgroups to the
        # 8 XCDs round-robin, then to the CUs of an XCD, then a second round
        # (P per CU): with the host's map word (launch + 20: bit 31 enable,
        # bits 0-7 log2 CUs per XCD, 8-15 P) workgroup w takes tile
        # (w % 8) * C * P + ((w / 8) % C) * P + w / (8 C): the P workgroups of
        # a CU take adjacent tiles and an XCD a contiguous block -- they share
        # pages (address translations) instead of each touching its own
        e("s_load_dword s99, s[8:9], 0x14")
        e("s_waitcnt lgkmcnt(0)")
        e("s_mov_b32 s16, s2")
        e("s_bitcmp1_b32 s99, 31")
        e("s_cbranch_scc0 .Lmap_done")
        e("s_bfe_u32 s97, s99, 0x80000")             # log2 C (bits 0-7)
        e("s_bfe_u32 s96, s99, 0x80008")             # P (bits 8-15; any value, e.g. 3)
        e("s_lshr_b32 s98, s2, 3")                   # r = w / 8
        e("s_bfm_b32 s95, s97, 0")                   # C - 1
        e("s_and_b32 s95, s98, s95")                 # cu = r % C
        e("s_lshr_b32 s98, s98, s97")                # slot = r / C
        e("s_mul_i32 s95, s95, s96")                 # cu * P
        e("s_add_u32 s98, s98, s95")                 # cu * P + slot
        e("s_lshl_b32 s95, s96, s97")                # C P
        e("s_and_b32 s16, s2, 7")
        e("s_mul_i32 s16, s16, s95")                 # (w % 8) C P
        e("s_add_u32 s16, s16, s98")
        self.label(".Lmap_done")
        e("s_mov_b32 s17, 0")
        e(f"v_mov_b32_e32 v{self.vSlot}, {self.dyn_lds()}")
        e("s_waitcnt vmcnt(0) lgkmcnt(0)")
        if self.PF:
            e("s_bitcmp1_b32 s100, 4")
            e("s_cbranch_scc1 .Lpf_start")
        if self.dbuf:
            # Software pipeline: while the ops run on tile i (registers A), tile
            # i+1 is already loading into registers B; at the top of iteration
            # i+1 B is copied to A.  Prologue: load the first tile into B.
            self.tile_check("s[16:17]", ".Ldone")
            self.base_of("s[16:17]", 68)
            self.wave_bytes(LD_WAVE, 70)
            if self.debug:
                # debug: record (wave id, tile, base, load byte offset, lane 0's
                # lane offset) per wave at debugBuf + 64 * (4 * wg + (s3 & 3))
                # and stop before touching the state
                e(f"s_load_dwordx2 s[94:95], s[8:9], {DEBUG_BUF}")     # debug buffer
                e("s_waitcnt lgkmcnt(0)")
                e("s_and_b32 s98, s3, 3")
                e("s_lshl_b32 s99, s2, 2")
                e("s_add_u32 s98, s98, s99")
                e("s_lshl_b32 s98, s98, 6")
                e("s_add_u32 s94, s94, s98")
                e("s_addc_u32 s95, s95, 0")
                vals = ["s3", "s16", "s17", "s68", "s69", "s96", "s97", "s2"]
                for k, sv in enumerate(vals):
                    e(f"v_mov_b32_e32 v{self.T[0] + (k % 8)}, {sv}")
                e(f"v_mov_b32_e32 v{self.T[4]}, 0")
                e("s_nop 1")
                e(f"v_cmp_eq_u32_e32 vcc, 0, v{vl}")
                e("s_and_saveexec_b64 s[98:99], vcc")
                e(f"global_store_dwordx4 v{self.T[4]}, v[{self.T[0]}:{self.T[0] + 3}], s[94:95]")
                e(f"global_store_dwordx4 v{self.T[4]}, v[{self.T[0] + 4}:{self.T[0] + 7}], s[94:95] offset:16")
                e(f"global_store_dword v{self.T[4]}, v{vldb}, s[94:95] offset:32")
                e("s_waitcnt vmcnt(0)")
                e("s_endpgm")
            self.groups("ld", 88, vldb, NG, self.B, 96)
            e("s_waitcnt vmcnt(0)")
            e("s_branch .Lcopy")
            self.label(".Ltile_loop")
            e(f"s_waitcnt vmcnt({2 * NG})")   # tile i+1's loads are older than tile i's stores
            self.label(".Lcopy")
            for r in range(0, 2 * self.P * NS, 2):
                e(f"v_mov_b64 v[{r}:{r + 1}], v[{self.B + r}:{self.B + r + 1}]")
            self.base_of("s[16:17]", 32)     # this tile: ctrlOut tests and stores
            # prefetch the next tile into B
            e("s_add_u32 s72, s16, s14")
            e("s_addc_u32 s73, s17, s15")
            self.tile_check("s[72:73]", ".Lno_prefetch")
            self.base_of("s[72:73]", 68)
            self.wave_bytes(LD_WAVE, 70)
            self.groups("ld", 88, vldb, NG, self.B, 96)
            self.label(".Lno_prefetch")
        else:
            # one tile at a time (latency hidden by the other waves of the SIMD)
            self.label(".Ltile_loop")
            self.tile_check("s[16:17]", ".Ldone")
            self.base_of("s[16:17]", 32)
            self.wave_bytes(LD_WAVE, 34)
            self.groups("ld", 88, vldb, NG, 0, 96)
            e("s_waitcnt vmcnt(0)")
            self.dyn_claim()
        # ---- op loop: prefetch op 0, then every op starts through next_op()
        self.label(".Lops_begin")
        e("s_mov_b64 s[94:95], s[10:11]")
        e("s_load_dwordx16 s[36:51], s[94:95], 0x0")
        self.label(".Lnext")
        self.next_op()
        self.check_path()
        self.label("wh_OPS_DONE")     # the sentinel record's handler
        self.handlers[LAYOUT["done"]] = "wh_OPS_DONE"
        e("s_waitcnt lgkmcnt(0)")      # the prefetch past the last op writes s[36:59]
        if self.PF:
            e("s_bitcmp1_b32 s100, 4")
            e("s_cbranch_scc1 .Lpf_end")
        if self.W:
            # store barrier (launch + 20, bit 30; set by the host for passes
            # whose store moves wave bits to other positions and that have no
            # wave-bit transposition): a wave's stores then land on addresses
            # other waves of the workgroup load, so every wave must have loaded
            # the tile (its loads completed before its first op) first
            e("s_load_dword s96, s[8:9], 0x14")
            e("s_waitcnt lgkmcnt(0)")
            e("s_bitcmp1_b32 s96, 30")
            e("s_cbranch_scc0 .Lst_nobar")
            e("s_barrier")
            self.label(".Lst_nobar")
        self.wave_bytes(ST_WAVE, 34)
        self.groups("st", 216, vstb, NG, 0, 96)
        if not self.dbuf:
            self.dyn_next(0 if self.nomem else 2 * NG)
        e("s_add_u32 s16, s16, s14")
        e("s_addc_u32 s17, s17, s15")
        if self.dbuf:
            self.tile_check("s[16:17]", ".Ldone")
        e("s_branch .Ltile_loop")
        self.label(".Ldone")
        e("s_endpgm")
        if self.PF:
            self.pf_paths(NG)
        # ---- handlers
        for kind in KINDS:
            for s in range(R):
                for c in (0, 1, 2):
                    self.gen_slot(kind, s, c)
        for s in range(R):
            for c in (0, 1, 2):
                self.gen_d2s(s, c)
        for c in (0, 1):
            self.gen_d2l(c)
        for creg in range(self.NS):
            for lane in (0, 1):
                self.gen_diag(creg, lane)
        for s in range(1, R):
            for l in range(6):
                self.gen_tr(s, l)
        for s in range(1, R):
            for b in range(self.W):
                self.gen_trw(s, b)
        for kind in LANE_KINDS:
            for l in range(LANE_BITS):
                for c in (0, 1):
                    self.gen_lane(kind, l, c)
        for kind in KINDS2:
            for s in range(R):
                for c in (0, 1, 2):
                    if kind == "HADD" and c:
                        continue   # only uncontrolled Hadamards drop their 1/sqrt2
                    self.gen_slot2(kind, s, c)
        for kind in CH_KINDS:
            for a in range(R):
                for b in range(R):
                    if a != b:
                        self.gen_ch(kind, a, b)
        for kind in PH_KINDS:
            for creg in range(NS):
                for lane in (0, 1):
                    self.gen_ph(kind, creg, lane)
        for lane, nt in ((0, R), (1, LANE_BITS if SWZ >= 2 else 0)):   # (lane variants: swizzle exchange only)
            for t in range(nt):
                for c in range(R):
                    if lane or c != t:
                        for v in (0, 1):
                            self.gen_swk(lane, t, c, v)
        self.finish_handler()
        L.append(".Lfunc_end0:")
        L.append("\t.size\tqa_wave_tile, .Lfunc_end0-qa_wave_tile")
        self.descriptor()

    def dyn_lds(self):
        """LDS byte address of the two tile-claim slots (after the outboxes)."""
        return self.NW * self.OUTBOX if (self.W or self.tr_lds) else 0

    def pf_lds(self):
        """LDS byte address of the prefetch areas (after the claim slots)."""
        return self.dyn_lds() + 16

    def pf_items(self, NG):
        """The tile's 16-byte loads per lane in groups() order: (jj, array
        SGPR pair, first VGPR); the last PF of them are prefetched."""
        out = []
        for jj in range(NG):
            out.append((jj, 4, 4 * jj))
            out.append((jj, 6, self.P * self.NS + 4 * jj))
        return out

    def pf_addr(self, Q, arr, bpair, jj):
        """Descriptor base of one 16-byte load / store: array + tile base
        (+ this wave's offset) + the group's offset (loaded to s[52:83] by
        half: groups 8h..8h+7 at s[52 + 16 slot]...)."""
        e = self.e
        g = 52 + 2 * (jj % 8) if self.pf_half_slot[jj // 8] == 0 else 68 + 2 * (jj % 8)
        e(f"s_add_u32 s{Q}, s{arr}, s{bpair}")
        e(f"s_addc_u32 s{Q + 1}, s{arr + 1}, s{bpair + 1}")
        e(f"s_add_u32 s{Q}, s{Q}, s{g}")
        e(f"s_addc_u32 s{Q + 1}, s{Q + 1}, s{g + 1}")

    def pf_vm(self, n=1):
        """Keep at most 63 vector-memory instructions in flight (the counter's
        range): a wait before an issue that could exceed it."""
        if self.pf_ub + n > 63:
            self.e(f"s_waitcnt vmcnt({63 - n})")
            self.pf_ub = 63 - n
        self.pf_ub += n

    def pf_paths(self, NG):
        """Looping grids with a next-tile prefetch (kernel argument bit 4 of a
        kernel generated with --pfa / --pfl).  Each workgroup runs tile t while
        tile t' = its next is already loading: at the top of tile t the last
        PF of t''s 16-byte loads per lane go to AGPRs / this wave's LDS area,
        the ops run, then t's stores go out -- each of the other groups'
        stores directly followed by the load of t''s group into the same
        registers -- and after one wait the prefetched groups are copied into
        place.  Claims: the first two tiles are the workgroup id and id +
        grid, later ones 2 grid + (counter value claimed one tile ahead)."""
        e = self.e
        items = self.pf_items(NG)
        n = len(items)
        P_from = n - self.PF
        pitems = [(k, items[k]) for k in range(P_from, n)]
        ditems = [(k, items[k]) for k in range(P_from)]
        # P item -> ("a", AGPR quad index) or ("l", LDS slot index)
        where = {}
        for i, (k, _) in enumerate(pitems):
            where[k] = ("a", i) if i < self.PFA else ("l", i - self.PFA)
        quads = (36, 40, 44, 48)

        def set_desc():
            for Q in quads:
                e(f"s_mov_b32 s{Q + 2}, -1")
                e(f"s_mov_b32 s{Q + 3}, 0x20000")

        def load_offsets(st_half, ld_half):
            # st / ld group offsets of half h into s[52:67] / s[68:83]
            self.pf_half_slot = {}
            if st_half is not None:
                e(f"s_load_dwordx16 s[52:67], s[8:9], {216 + 64 * st_half}")
            if ld_half is not None:
                e(f"s_load_dwordx16 s[68:83], s[8:9], {88 + 64 * ld_half}")
            e("s_waitcnt lgkmcnt(0)")

        # ---- start: the first tile loads directly
        self.label(".Lpf_start")
        e("s_add_u32 s0, s16, s14")                     # t' = first tile + grid
        e(f"s_mul_i32 s1, s3, {self.PFL * 1024}")
        e(f"s_add_u32 s1, s1, {self.pf_lds()}")          # this wave's LDS prefetch area
        e(f"v_lshlrev_b32_e32 v{self.vPF}, 4, v{self.vLane}")
        e(f"v_add_u32_e32 v{self.vPF}, s1, v{self.vPF}")
        self.tile_check("s[16:17]", ".Ldone")
        self.base_of("s[16:17]", 32)
        self.wave_bytes(LD_WAVE, 34)
        self.groups("ld", 88, self.vLdB, NG, 0, 96)
        e("s_waitcnt vmcnt(0)")
        # ---- top of tile t: claim t'' and prefetch t''s last PF loads
        self.label(".Lpf_top")
        self.base_of("s[16:17]", 32)                    # this tile: ctrlOut tests and stores
        e("s_sub_u32 s98, s0, s12")
        e("s_subb_u32 s99, 0, s13")
        e("s_cbranch_scc0 .Lops_begin")                 # no t': nothing to claim or prefetch
        self.pf_ub = self.PF                            # the previous tile's prefetched groups' stores
        self.pf_vm()
        self.dyn_claim()
        e("s_mov_b32 s84, s0")
        e("s_mov_b32 s85, 0")
        self.base_of("s[84:85]", 84)
        self.wave_bytes(LD_WAVE, 86)                    # s[96:97]: t''s bytes + this wave's
        halves = sorted({jj // 8 for _, (jj, _, _) in pitems})
        set_desc()
        q = 0
        for h in halves:
            load_offsets(None, h)
            self.pf_half_slot = {h: 1}
            for k, (jj, arr, vb) in pitems:
                if jj // 8 != h:
                    continue
                Q = quads[q % 4]
                q += 1
                self.pf_addr(Q, arr, 96, jj)
                self.pf_vm()
                kind, i = where[k]
                if kind == "a":
                    e(f"buffer_load_dwordx4 a[{4 * i}:{4 * i + 3}], v{self.vLdB}, s[{Q}:{Q + 3}], 0 offen{LD_POLICY}")
                else:
                    e(f"s_add_u32 m0, s1, {1024 * i}")
                    e(f"buffer_load_dwordx4 v{self.vLdB}, s[{Q}:{Q + 3}], 0 offen{LD_POLICY} lds")
        e("s_branch .Lops_begin")
        # ---- end of tile t
        self.label(".Lpf_end")
        if self.W:
            e("s_load_dword s96, s[8:9], 0x14")
            e("s_waitcnt lgkmcnt(0)")
            e("s_bitcmp1_b32 s96, 30")
            e("s_cbranch_scc0 .Lpf_nobar")
            e("s_barrier")
            self.label(".Lpf_nobar")
        e("s_waitcnt vmcnt(0)")                         # t''s prefetch and the claim have landed
        self.pf_ub = 0
        e("s_sub_u32 s98, s0, s12")
        e("s_subb_u32 s99, 0, s13")
        e("s_cbranch_scc1 .Lpf_more")
        # the workgroup's last tile: plain stores
        self.wave_bytes(ST_WAVE, 34)
        self.groups("st", 216, self.vStB, NG, 0, 96)
        e("s_endpgm")
        self.label(".Lpf_more")
        e("s_mov_b32 s84, s0")
        e("s_mov_b32 s85, 0")
        self.base_of("s[84:85]", 84)
        e("s_lshl_b32 s98, s3, 3")
        e(f"s_add_u32 s98, s98, {LD_WAVE}")
        e("s_load_dwordx2 s[88:89], s[8:9], s98 offset:0x0")
        e("s_waitcnt lgkmcnt(0)")
        e("s_add_u32 s88, s88, s86")                    # s[88:89]: t''s bytes + this wave's
        e("s_addc_u32 s89, s89, s87")
        self.wave_bytes(ST_WAVE, 34)                    # s[96:97]: t's store bytes + this wave's
        set_desc()
        q = 0
        # the other groups: store, then t''s load into the same registers
        for h in sorted({jj // 8 for _, (jj, _, _) in ditems}):
            load_offsets(h, h)
            self.pf_half_slot = {h: 0}
            for k, (jj, arr, vb) in ditems:
                if jj // 8 != h:
                    continue
                Q = quads[q % 4]
                q += 1
                self.pf_addr(Q, arr, 96, jj)
                self.pf_vm()
                e(f"buffer_store_dwordx4 v[{vb}:{vb + 3}], v{self.vStB}, s[{Q}:{Q + 3}], 0 offen{ST_POLICY}")
                Q = quads[q % 4]
                q += 1
                self.pf_half_slot = {h: 1}
                self.pf_addr(Q, arr, 88, jj)
                self.pf_half_slot = {h: 0}
                self.pf_vm()
                e(f"buffer_load_dwordx4 v[{vb}:{vb + 3}], v{self.vLdB}, s[{Q}:{Q + 3}], 0 offen{LD_POLICY}")
        # the prefetched groups: stores only (the last VMEM instructions)
        for h in halves:
            load_offsets(h, None)
            self.pf_half_slot = {h: 0}
            for k, (jj, arr, vb) in pitems:
                if jj // 8 != h:
                    continue
                Q = quads[q % 4]
                q += 1
                self.pf_addr(Q, arr, 96, jj)
                self.pf_vm()
                e(f"buffer_store_dwordx4 v[{vb}:{vb + 3}], v{self.vStB}, s[{Q}:{Q + 3}], 0 offen{ST_POLICY}")
        e(f"s_waitcnt vmcnt({self.PF})")                # t''s direct loads (and everything older) landed
        # publish the claim (wave 0), take it after the barrier (which also
        # orders the LDS prefetch for the reads below)
        e("s_cmp_eq_u32 s3, 0")
        e("s_cbranch_scc0 .Lpf_bar")
        e("s_mov_b64 s[98:99], exec")
        e("s_mov_b64 exec, 1")
        e(f"ds_write_b32 v{self.vSlot}, v{self.vNext}")
        e("s_mov_b64 exec, s[98:99]")
        self.label(".Lpf_bar")
        e("s_waitcnt lgkmcnt(0)")
        e("s_barrier")
        e(f"ds_read_b32 v{self.vNext}, v{self.vSlot}")
        e(f"v_xor_b32_e32 v{self.vSlot}, 4, v{self.vSlot}")
        e("s_nop 1")
        for k, (jj, arr, vb) in pitems:
            kind, i = where[k]
            if kind == "a":
                for x in range(4):
                    e(f"v_accvgpr_read_b32 v{vb + x}, a{4 * i + x}")
            else:
                e(f"ds_read_b128 v[{vb}:{vb + 3}], v{self.vPF} offset:{1024 * i}")
        e("s_waitcnt lgkmcnt(0)")
        e(f"v_readfirstlane_b32 s94, v{self.vNext}")
        e("s_nop 4")
        e("s_mov_b32 s16, s0")
        e("s_mov_b32 s17, 0")
        e("s_lshl_b32 s0, s14, 1")
        e("s_add_u32 s0, s0, s94")                      # t'' = 2 grid + its claim
        e("s_branch .Lpf_top")

    def dyn_claim(self):
        """Looping grids with dynamic claims (kernel argument bit 4): wave 0's
        lane 0 claims the workgroup's next tile now -- an atomic add on the
        launch's counter (bits 5-7 pick it) that returns during the ops.  A
        static stride would give each workgroup tiles with the same low index
        bits, and with them the same out-of-tile controls: some workgroups
        would run every controlled op and others none (persistent grids ran
        18 % slower than one-tile grids on compute alone)."""
        e = self.e
        self.dyn_label = getattr(self, "dyn_label", 0) + 1
        skip = f".Ldyn_claim_{self.dyn_label}"
        e("s_bitcmp1_b32 s100, 4")
        e(f"s_cbranch_scc0 {skip}")
        e("s_cmp_eq_u32 s3, 0")
        e(f"s_cbranch_scc0 {skip}")
        e("s_bfe_u32 s96, s100, 0x30005")             # counter index (bits 5-7)
        e("s_lshl_b32 s96, s96, 2")
        e(f"s_add_u32 s96, s96, {TILE_CNT}")
        e("s_add_u32 s96, s8, s96")
        e("s_addc_u32 s97, s9, 0")
        e(f"v_mov_b32_e32 v{self.vNext}, 1")
        e("s_mov_b64 s[98:99], exec")
        e("s_mov_b64 exec, 1")
        # (vLane is 0 in lane 0: the counter's own address)
        e(f"global_atomic_add v{self.vNext}, v{self.vLane}, v{self.vNext}, s[96:97] sc0")
        e("s_mov_b64 exec, s[98:99]")
        self.label(skip)

    def dyn_next(self, newer):
        """End of a tile with dynamic claims: wave 0 publishes its claim
        through LDS (two slots used alternately, so a wave that runs a tile
        ahead cannot overwrite a slot another wave has yet to read), every
        wave of the workgroup takes it after a barrier and continues with tile
        waveStride + claim.  `newer`: VMEM instructions issued after the claim
        (the tile's stores), which its wait leaves in flight."""
        e = self.e
        static, bar = ".Ldyn_static", ".Ldyn_bar"
        e("s_bitcmp1_b32 s100, 4")
        e(f"s_cbranch_scc0 {static}")
        e("s_cmp_eq_u32 s3, 0")
        e(f"s_cbranch_scc0 {bar}")
        e(f"s_waitcnt vmcnt({newer})")
        e("s_mov_b64 s[98:99], exec")
        e("s_mov_b64 exec, 1")
        e(f"ds_write_b32 v{self.vSlot}, v{self.vNext}")
        e("s_mov_b64 exec, s[98:99]")
        self.label(bar)
        e("s_waitcnt lgkmcnt(0)")
        e("s_barrier")
        e(f"ds_read_b32 v{self.vNext}, v{self.vSlot}")
        e(f"v_xor_b32_e32 v{self.vSlot}, 4, v{self.vSlot}")
        e("s_waitcnt lgkmcnt(0)")
        e(f"v_readfirstlane_b32 s16, v{self.vNext}")
        e("s_nop 4")                          # VALU-written SGPR read by SALU
        e("s_add_u32 s16, s16, s14")
        e("s_mov_b32 s17, 0")
        e("s_branch .Ltile_loop")
        self.label(static)

    def tile_check(self, tile, done):
        """Branch to `done` unless tile < numTiles (s[12:13])."""
        lo = int(tile[2:tile.index(":")])
        self.e(f"s_sub_u32 s98, s{lo}, s12")
        self.e(f"s_subb_u32 s99, s{lo + 1}, s13")
        self.e(f"s_cbranch_scc0 {done}")

    def wave_bytes(self, off, bpair):
        """s[96:97] = s[bpair:bpair+1] + this wave's byte offset (launch record
        + off + 8 * wave): the tile bits on wave bits are uniform per wave."""
        e = self.e
        if not self.W:
            e(f"s_mov_b64 s[96:97], s[{bpair}:{bpair + 1}]")
            return
        e("s_lshl_b32 s98, s3, 3")
        e(f"s_add_u32 s98, s98, {off}")
        e("s_load_dwordx2 s[96:97], s[8:9], s98 offset:0x0")   # SGPR offset, SOE form
        e("s_waitcnt lgkmcnt(0)")
        e(f"s_add_u32 s96, s96, s{bpair}")
        e(f"s_addc_u32 s97, s97, s{bpair + 1}")

    def insert_bits(self, d):
        """Split launches (a pass run on one part of the state while a qubit
        swap moves the others, src/hip/backend_hip.hip): kernel argument s100
        = n (bits 0-1) insertions of bit value v_m (bit 14 + 8m) at tile-index
        bit j_m (bits 8 + 8m .. 13 + 8m), ascending j -- the launch's tile t
        becomes the t-th tile whose index has those bits.  n = 0: all tiles."""
        e = self.e
        self.ins_label = getattr(self, "ins_label", 0) + 1
        done = f".Lins_done_{self.ins_label}"
        e("s_and_b32 s101, s100, 3")
        for m in range(3):
            e(f"s_cmp_le_u32 s101, {m}")
            e(f"s_cbranch_scc1 {done}")
            e(f"s_bfe_u32 s94, s100, {(6 << 16) | (8 + 8 * m):#x}")      # j
            e("s_bfm_b64 s[96:97], s94, 0")                               # 2^j - 1
            e(f"s_and_b64 s[98:99], s[{d}:{d + 1}], s[96:97]")
            e(f"s_lshr_b64 s[{d}:{d + 1}], s[{d}:{d + 1}], s94")
            e("s_add_u32 s95, s94, 1")
            e(f"s_lshl_b64 s[{d}:{d + 1}], s[{d}:{d + 1}], s95")
            e(f"s_or_b64 s[{d}:{d + 1}], s[{d}:{d + 1}], s[98:99]")
            e(f"s_bitcmp1_b32 s100, {14 + 8 * m}")                        # v
            e(f"s_cbranch_scc0 .Lins_zero_{self.ins_label}_{m}")
            e("s_bfm_b64 s[96:97], 1, s94")
            e(f"s_or_b64 s[{d}:{d + 1}], s[{d}:{d + 1}], s[96:97]")
            self.label(f".Lins_zero_{self.ins_label}_{m}")
        self.label(done)

    def tile_order(self, d):
        """Experiment (QUEST_WAVE_TILE_ORDER, bits 2-3 of the launch argument
        s100): the order in which the launch's tiles are dealt to workgroups.
        0: tile = index; 1: bit-reversed index (workgroups running together
        differ in the HIGH non-tile positions); 2: XCD blocks (index i takes
        tile (i % 8) * T / 8 + i / 8: the workgroups an XCD runs together take
        adjacent tiles of its own eighth).  T = the launch's tile count (a power
        of two, >= 8, else the order stays 0)."""
        e = self.e
        self.ord_label = getattr(self, "ord_label", 0) + 1
        done, blk = f".Lord_done_{self.ord_label}", f".Lord_blk_{self.ord_label}"
        e("s_bfe_u32 s94, s100, 0x20002")             # order (bits 2-3)
        e("s_cmp_eq_u32 s94, 0")
        e(f"s_cbranch_scc1 {done}")
        e("s_ff1_i32_b32 s95, s12")                   # log2 T
        e("s_cmp_lt_u32 s95, 3")
        e(f"s_cbranch_scc1 {done}")
        e("s_cmp_eq_u32 s94, 1")
        e(f"s_cbranch_scc0 {blk}")
        e(f"s_brev_b32 s{d}, s{d}")
        e("s_sub_u32 s94, 32, s95")
        e(f"s_lshr_b32 s{d}, s{d}, s94")
        e(f"s_branch {done}")
        self.label(blk)
        e(f"s_and_b32 s94, s{d}, 7")
        e("s_sub_u32 s98, s95, 3")
        e("s_lshl_b32 s94, s94, s98")
        e(f"s_lshr_b32 s{d}, s{d}, 3")
        e(f"s_or_b32 s{d}, s{d}, s94")
        self.label(done)

    def base_of(self, tile, d):
        """s[d:d+1] = tile index with zeros inserted at pos[0..K-1] (ascending),
        s[d+2:d+3] = the same in bytes."""
        e = self.e
        e(f"s_mov_b64 s[{d}:{d + 1}], {tile}")
        self.tile_order(d)
        self.insert_bits(d)
        K = self.R + 6 + self.W
        assert K <= 24, "pos[] lives in s[20:31] (b >= 12 in bits 8..)"
        for b in range(K):
            p = f"s{20 + b}"
            if b >= 12:   # the s_*64 shift / bfm operands use bits 5:0 only
                e(f"s_lshr_b32 s95, s{20 + b - 12}, 8")   # s[94:95] is free outside the op loop
                p = "s95"
            e(f"s_bfm_b64 s[96:97], {p}, 0")
            e(f"s_and_b64 s[98:99], s[{d}:{d + 1}], s[96:97]")
            e(f"s_lshr_b64 s[{d}:{d + 1}], s[{d}:{d + 1}], {p}")
            e(f"s_add_u32 s94, {p}, 1")
            e(f"s_lshl_b64 s[{d}:{d + 1}], s[{d}:{d + 1}], s94")
            e(f"s_or_b64 s[{d}:{d + 1}], s[{d}:{d + 1}], s[98:99]")
        e(f"s_lshl_b64 s[{d + 2}:{d + 3}], s[{d}:{d + 1}], {3 if self.P == 2 else 2}")   # bytes

    def groups(self, what, off, vb, NG, regbase, bpair):
        """Load or store the NG 16-byte groups of re and im (per lane) of the
        register set at `regbase`, tile base in bytes in s[bpair:bpair+1]."""
        e = self.e
        prio = getattr(self, "setprio", False) and not self.nomem
        if prio:
            e("s_setprio 2")   # issue this tile's memory ahead of the other waves' arithmetic
        # group byte offsets, 8 per s_load_dwordx16
        for half in range(0, NG, 8):
            n = min(8, NG - half)
            dst = 52 if half == 0 else 68
            e(f"s_load_dwordx16 s[{dst}:{dst + 15}], s[8:9], {off + 8 * half}")
        # descriptor words 2,3 of the four quads (s[36:59] also holds the
        # prefetched op record during the op loop)
        for Q in (36, 40, 44, 48):
            e(f"s_mov_b32 s{Q + 2}, -1")
            e(f"s_mov_b32 s{Q + 3}, 0x20000")
        e("s_waitcnt lgkmcnt(0)")
        q = 0
        for jj in range(NG):
            g = (52 + 2 * jj) if jj < 8 else (68 + 2 * (jj - 8))
            for arr, base in ((4, regbase + 4 * jj), (6, regbase + self.P * self.NS + 4 * jj)):
                Q = (36, 40, 44, 48)[q % 4]
                q += 1
                e(f"s_add_u32 s{Q}, s{arr}, s{bpair}")
                e(f"s_addc_u32 s{Q + 1}, s{arr + 1}, s{bpair + 1}")
                e(f"s_add_u32 s{Q}, s{Q}, s{g}")
                e(f"s_addc_u32 s{Q + 1}, s{Q + 1}, s{g + 1}")
                if self.nomem:
                    continue
                if what == "ld":
                    e(f"buffer_load_dwordx4 v[{base}:{base + 3}], v{vb}, s[{Q}:{Q + 3}], 0 offen{LD_POLICY}")
                    for _ in range(LD_PACE):
                        e("s_nop 3")
                else:
                    e(f"buffer_store_dwordx4 v[{base}:{base + 3}], v{vb}, s[{Q}:{Q + 3}], 0 offen{ST_POLICY}")
        if prio:
            e("s_setprio 0")

    def descriptor(self):
        nv = self.nvgpr
        nv8 = (nv + 7) // 8 * 8
        accum, nagpr = nv8, 0
        if self.PF and self.PFA:
            # unified register file: AGPRs after the architectural VGPRs
            accum = (nv + 3) // 4 * 4
            nagpr = 4 * self.PFA
            nv8 = (accum + nagpr + 7) // 8 * 8
        L = self.lines
        L.append("\t.section\t.rodata,\"a\",@progbits")
        L.append("\t.p2align\t6, 0x0")
        L.append("\t.amdhsa_kernel qa_wave_tile")
        lds = self.pf_lds() + (self.NW * self.PFL * 1024 if self.PF else 0)   # outboxes, claim slots, prefetch
        for k, v in [("group_segment_fixed_size", lds), ("private_segment_fixed_size", 0), ("kernarg_size", 32),
                     ("user_sgpr_count", 2), ("user_sgpr_dispatch_ptr", 0), ("user_sgpr_queue_ptr", 0),
                     ("user_sgpr_kernarg_segment_ptr", 1), ("user_sgpr_dispatch_id", 0),
                     ("user_sgpr_kernarg_preload_length", 0), ("user_sgpr_kernarg_preload_offset", 0),
                     ("user_sgpr_private_segment_size", 0), ("uses_dynamic_stack", 0),
                     ("enable_private_segment", 0), ("system_sgpr_workgroup_id_x", 1),
                     ("system_sgpr_workgroup_id_y", 0), ("system_sgpr_workgroup_id_z", 0),
                     ("system_sgpr_workgroup_info", 0), ("system_vgpr_workitem_id", 0),
                     ("next_free_vgpr", nv8), ("next_free_sgpr", 102), ("accum_offset", accum),
                     ("reserve_vcc", 1), ("float_round_mode_32", 0), ("float_round_mode_16_64", 0),
                     ("float_denorm_mode_32", 3), ("float_denorm_mode_16_64", 3), ("dx10_clamp", 1),
                     ("ieee_mode", 1), ("fp16_overflow", 0), ("tg_split", 0)]:
            L.append(f"\t\t.amdhsa_{k} {v}")
        L.append("\t.end_amdhsa_kernel")
        L.append("\t.text")
        L.append("\t.p2alignl 6, 3212836864")
        L.append("\t.fill 256, 4, 3212836864")
        L.append("\t.amdgpu_metadata")
        L.append(f"""---
amdhsa.kernels:
  - .agpr_count:     {nagpr}
    .args:
      - .address_space:  global
        .offset:         0
        .size:           8
        .value_kind:     global_buffer
      - .address_space:  global
        .offset:         8
        .size:           8
        .value_kind:     global_buffer
      - .address_space:  global
        .offset:         16
        .size:           8
        .value_kind:     global_buffer
      - .offset:         24
        .size:           4
        .value_kind:     by_value
    .group_segment_fixed_size: {lds}
    .kernarg_segment_align: 8
    .kernarg_segment_size: 32
    .language:       OpenCL C
    .language_version:
      - 2
      - 0
    .max_flat_workgroup_size: {64 * self.NW}
    .name:           qa_wave_tile
    .private_segment_fixed_size: 0
    .sgpr_count:     104
    .sgpr_spill_count: 0
    .symbol:         qa_wave_tile.kd
    .uniform_work_group_size: 1
    .uses_dynamic_stack: false
    .vgpr_count:     {nv8}
    .vgpr_spill_count: 0
    .wavefront_size: 64
amdhsa.target:   amdgcn-amd-amdhsa--gfx950
amdhsa.version:
  - 1
  - 2
...""")
        L.append("\t.end_amdgpu_metadata")


def elf_symbols(path):
    """name -> value of the symbols of an ELF64 relocatable/shared object."""
    data = open(path, "rb").read()
    assert data[:4] == b"\x7fELF" and data[4] == 2
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    secs = []
    for k in range(shnum):
        name, typ, flags, addr, off, size, link, info, align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", data, shoff + k * shentsize)
        secs.append((name, typ, off, size, link, entsize))
    out = {}
    for name, typ, off, size, link, entsize in secs:
        if typ != 2:  # SHT_SYMTAB
            continue
        stroff = secs[link][2]
        for k in range(size // entsize):
            st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", data,
                                                                                          off + k * entsize)
            end = data.index(b"\0", stroff + st_name)
            out[data[stroff + st_name:end].decode()] = st_value
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["asm", "embed"])
    ap.add_argument("--slots", type=int, default=4)
    ap.add_argument("--prec", type=int, default=2, choices=[1, 2], help="QuEST_PREC: 2 fp64, 1 fp32")
    ap.add_argument("--dbuf", type=int, default=-1, help="software-pipelined tiles (default: when 4 slots)")
    ap.add_argument("--wbits", type=int, default=3, help="2^wbits waves share a tile")
    ap.add_argument("--debug", action="store_true", help="record addressing state per wave and stop (no state access)")
    ap.add_argument("--nomem", action="store_true", help="experiment: drop the state loads and stores")
    ap.add_argument("--setprio", action="store_true",
                    help="experiment: raise the wave priority while issuing a tile's loads / stores")
    ap.add_argument("--lean", type=int, default=0, help="1: 80-VGPR layout, half outboxes (3 workgroups per CU)")
    ap.add_argument("--pfa", type=int, default=0, help="next-tile prefetch: 16-byte loads per lane into AGPRs")
    ap.add_argument("--pfl", type=int, default=0, help="next-tile prefetch: 16-byte loads per lane into LDS")
    ap.add_argument("--out", required=True)
    ap.add_argument("--obj")
    ap.add_argument("--hsaco")
    args = ap.parse_args()
    if args.mode == "asm":
        # the second register set costs a wave per SIMD: worth it only while
        # a tile has <= 4 waves (otherwise too few workgroups fit a CU)
        dbuf = args.dbuf if args.dbuf >= 0 else (args.slots <= 4 and args.wbits <= 2)
        set_layout(args.slots)
        g = Gen(args.slots, dbuf, args.wbits, 2 if args.prec == 2 else 1, args.debug, args.nomem, bool(args.lean),
                args.pfa, args.pfl)
        g.setprio = args.setprio
        g.kernel()
        with open(args.out, "w") as f:
            f.write("// GENERATED by tools/gen_wave_asm.py -- do not edit\n")
            f.write(f"// wave_prefetch {g.PF}\n")
            f.write("\n".join(g.lines) + "\n")
        # handler names per table index, for the embed step
        with open(args.out + ".handlers", "w") as f:
            for i in range(table_size(args.slots)):
                f.write(f"{i} {g.handlers.get(i, '-')}\n")
        return
    syms = elf_symbols(args.obj)
    anchor = syms["qa_wave_tile"]
    table = []
    for line in open(args.out.replace("wave_image.inc", "wave_kernel.s") + ".handlers"):
        i, name = line.split()
        table.append(syms[name] - anchor if name != "-" else 0)
    img = open(args.hsaco, "rb").read()
    with open(args.out, "w") as f:
        f.write("// GENERATED by tools/gen_wave_asm.py embed -- do not edit\n")
        f.write(f"static const int kWaveImageSlots = {args.slots};\n")
        f.write(f"static const int kWaveImageWBits = {args.wbits};\n")
        src = open(args.out.replace("wave_image.inc", "wave_kernel.s")).read()
        vg = re.search(r"amdhsa_next_free_vgpr (\d+)", src)
        f.write(f"static const int kWaveImageVgprs = {vg.group(1)};\n")
        lds = int(re.search(r"amdhsa_group_segment_fixed_size (\d+)", src).group(1))
        pf = int(re.search(r"// wave_prefetch (\d+)", src).group(1))
        # resident workgroups per CU (512 registers per SIMD lane, 160 KiB LDS;
        # a workgroup of 2^wbits waves puts 2^wbits / 4 of them on each SIMD)
        per_simd = 512 // int(vg.group(1))
        wg = min(per_simd * 4 // (1 << args.wbits), (160 * 1024) // max(1, lds))
        f.write(f"static const int kWaveImagePrefetch = {pf};\n")
        f.write(f"static const int kWaveImageWgPerCU = {max(1, wg)};\n")
        set_layout(args.slots)
        f.write(f"static const int kWaveImagePrec = {args.prec};\n")
        for k in ("slot", "d2s", "d2l", "tr", "diag", "trw", "lane", "slot2", "ph", "ch", "slotL", "slot2L", "d2sL", "swk", "check"):
            f.write(f"static const int kWaveIdx_{k} = {LAYOUT[k]};\n")
        f.write(f"static const int kWaveSentinelIndex = {LAYOUT['done']};\n")
        f.write(f"static const int kWaveHandlerOffset[{len(table)}] = {{{', '.join(map(str, table))}}};\n")
        f.write(f"static const unsigned char kWaveImage[{len(img)}] __attribute__((aligned(4096))) = {{\n")
        for k in range(0, len(img), 24):
            f.write(", ".join(str(b) for b in img[k:k + 24]) + ",\n")
        f.write("};\n")


if __name__ == "__main__":
    main()
