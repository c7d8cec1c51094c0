"""Assembler for GPU_ACTOR_HT_PROGRAM types: behaviours given at run time
(include/gpu_actor.h, gpu_actor_type_program) instead of a compiled handler
table — the reference's generated dispatch (src/libponyc/codegen/gentype.c:
358-395) for any behaviour set, without rebuilding the library.

    p = Program()
    p.behaviour(0)                  # code of behaviour 0 starts here
    p.addi(0, 0, 1)                 # r0 (state word 0) += 1
    p.send(9, 0, 8)                 # send behaviour 0, arg r8, to r9 (self)
    p.halt()
    eng.type_register(t, 8, HT_PROGRAM); eng.type_program(t, p.assemble())

Registers: r0-r7 the state words, r8 the argument, r9 the actor's id, r10 the
behaviour, r11-r15 zero at entry. Jumps take label names."""
from __future__ import annotations

import numpy as np

ENTRIES = 16
MAX_STEPS = 4096
OPS = {"halt": 0, "ldi": 1, "ldp": 2, "mov": 3, "add": 4, "sub": 5, "mul": 6, "mulhi": 7,
       "and": 8, "or": 9, "xor": 10, "shl": 11, "shr": 12, "addi": 13, "ltu": 14, "eq": 15,
       "jz": 16, "jnz": 17, "jmp": 18, "send": 19, "mix": 20, "yield": 21, "spawn": 22}
R_ARG, R_SELF, R_BEH = 8, 9, 10


def word(op: int, d: int = 0, a: int = 0, b: int = 0, imm: int = 0) -> int:
    """One instruction: op | d << 8 | a << 12 | b << 16 | (uint32)imm << 32."""
    if not (-(1 << 31) <= imm < (1 << 32)):
        raise ValueError(f"immediate {imm} does not fit 32 bits")
    for r in (d, a, b):
        if not 0 <= r < 16:
            raise ValueError(f"register {r}")
    return op | d << 8 | a << 12 | b << 16 | (imm & 0xFFFFFFFF) << 32


class Program:
    def __init__(self):
        self.code: list = []            # words, or (op, d, a, b, label) for jumps
        self.entries = [0] * ENTRIES
        self.labels: dict = {}

    def behaviour(self, beh: int) -> None:
        self.entries[beh] = ENTRIES + len(self.code)

    def label(self, name: str) -> None:
        self.labels[name] = len(self.code)

    def _op(self, name, d=0, a=0, b=0, imm=0):
        self.code.append(word(OPS[name], d, a, b, imm))

    def _jump(self, name, a, label):
        self.code.append((OPS[name], a, label))

    # r[d] = ...
    def ldi(self, d, imm): self._op("ldi", d, imm=imm)
    def ldp(self, d, k): self._op("ldp", d, imm=k)
    def mov(self, d, a): self._op("mov", d, a)
    def add(self, d, a, b): self._op("add", d, a, b)
    def sub(self, d, a, b): self._op("sub", d, a, b)
    def mul(self, d, a, b): self._op("mul", d, a, b)
    def mulhi(self, d, a, b): self._op("mulhi", d, a, b)
    def and_(self, d, a, b): self._op("and", d, a, b)
    def or_(self, d, a, b): self._op("or", d, a, b)
    def xor(self, d, a, b): self._op("xor", d, a, b)
    def shl(self, d, a, b): self._op("shl", d, a, b)
    def shr(self, d, a, b): self._op("shr", d, a, b)
    def addi(self, d, a, imm): self._op("addi", d, a, imm=imm)
    def ltu(self, d, a, b): self._op("ltu", d, a, b)
    def eq(self, d, a, b): self._op("eq", d, a, b)
    def mix(self, d, a): self._op("mix", d, a)
    # control, effects
    def jz(self, a, label): self._jump("jz", a, label)
    def jnz(self, a, label): self._jump("jnz", a, label)
    def jmp(self, label): self._jump("jmp", 0, label)
    def send(self, to, beh, arg): self._op("send", 0, to, arg, imm=beh)
    def spawn(self, type_id, beh, arg):
        """pony_create of an actor of type `type_id` + its constructor message
        (behaviour `beh`, argument r[arg]); its id is assigned when the step ends."""
        if not (0 <= type_id < 256 and 0 <= beh < 16):
            raise ValueError("spawn type < 256, behaviour < 16")
        self._op("spawn", 0, 0, arg, imm=type_id | beh << 8)
    def yield_(self): self._op("yield")
    def halt(self): self._op("halt")
    def raw(self, w: int) -> None:
        self.code.append(int(w) & 0xFFFFFFFFFFFFFFFF)

    def assemble(self) -> np.ndarray:
        out = list(self.entries)
        for pc, c in enumerate(self.code):
            if isinstance(c, tuple):
                op, a, label = c
                out.append(word(op, 0, a, 0, self.labels[label] - (pc + 1)))
            else:
                out.append(c)
        return np.array(out, dtype=np.uint64)


# ---- the examples' behaviours as programs (parity against the compiled tables) ----
def ring_program() -> np.ndarray:
    """examples/ring/main.pony:13-24 (the compiled GPU_ACTOR_HT_RING): word 0
    the next actor, 2 passes received, 3 rings finished here."""
    p = Program()
    p.behaviour(0)                      # set(next)
    p.mov(0, R_ARG)
    p.halt()
    p.behaviour(1)                      # pass(i)
    p.addi(2, 2, 1)
    p.jz(R_ARG, "done")
    p.ldi(11, -1)                       # GPU_ACTOR_NONE
    p.eq(12, 0, 11)
    p.jnz(12, "end")
    p.addi(13, R_ARG, -1)
    p.send(0, 1, 13)
    p.halt()
    p.label("done")
    p.addi(3, 3, 1)
    p.label("end")
    p.halt()
    return p.assemble()


def det_program(beh: int = 0) -> np.ndarray:
    """The deterministic message-ubench ping (the compiled
    GPU_ACTOR_HT_PINGER_DET, engine_dev.h det_ping): count += 1; acc ^= arg;
    below the hop limit (param 2) forward to param 1 + mulhi(mix(param 3 ^
    arg), param 0) with the hop count + 1."""
    p = Program()
    p.behaviour(beh)
    p.addi(0, 0, 1)
    p.xor(1, 1, R_ARG)
    p.ldi(11, 32)
    p.ldi(12, -1)
    p.shr(12, 12, 11)                   # 0xFFFFFFFF
    p.and_(13, R_ARG, 12)               # hop
    p.ldp(14, 2)
    p.ltu(15, 13, 14)
    p.jz(15, "end")
    p.ldp(14, 3)
    p.xor(14, 14, R_ARG)
    p.mix(14, 14)
    p.ldp(15, 0)
    p.mulhi(14, 14, 15)
    p.ldp(15, 1)
    p.add(14, 14, 15)                   # the receiver
    p.addi(13, 13, 1)
    p.shl(15, 12, 11)                   # 0xFFFFFFFF00000000
    p.and_(15, R_ARG, 15)
    p.or_(15, 15, 13)
    p.send(14, beh, 15)
    p.label("end")
    p.halt()
    return p.assemble()


def spreader_program(type_id: int) -> np.ndarray:
    """examples/spreader/main.pony:1-48 (the compiled GPU_ACTOR_HT_SPREADER,
    engine_dev.h) for a program type `type_id`: word 0 count, 1 parent (~0:
    the root), 2 _result, 3 _received, 4 the root's printed total.
    Behaviour 0 SPREAD(parent << 32 | count) — the constructor — spawns two
    children of its own type when count > 1 (SPAWN); behaviour 1 RESULT(i)."""
    p = Program()
    p.behaviour(0)                      # new create / new spread
    p.ldi(11, 32)
    p.ldi(12, -1)                       # GPU_ACTOR_NONE
    p.shr(13, 12, 11)                   # 0xFFFFFFFF
    p.and_(0, R_ARG, 13)                # count
    p.shr(14, R_ARG, 11)                # parent
    p.mov(1, 14)
    p.eq(15, 14, 13)
    p.jz(15, "has_parent")
    p.mov(1, 12)                        # the root: parent = NONE
    p.label("has_parent")
    p.ldi(15, 2)
    p.ltu(15, 0, 15)                    # count <= 1
    p.jz(15, "spawn")
    p.eq(15, 1, 12)
    p.jnz(15, "root_leaf")
    p.ldi(14, 1)
    p.send(1, 1, 14)                    # RESULT(1) to the parent
    p.halt()
    p.label("root_leaf")
    p.ldi(4, 1)                         # "1 actor"
    p.halt()
    p.label("spawn")
    p.shl(14, R_SELF, 11)
    p.addi(15, 0, -1)
    p.or_(14, 14, 15)                   # self << 32 | count - 1
    p.spawn(type_id, 0, 14)
    p.spawn(type_id, 0, 14)
    p.halt()
    p.behaviour(1)                      # be result(i)
    p.addi(3, 3, 1)
    p.add(2, 2, R_ARG)
    p.ldi(15, 2)
    p.eq(15, 3, 15)
    p.jz(15, "wait")
    p.addi(14, 2, 1)
    p.ldi(12, -1)
    p.eq(15, 1, 12)
    p.jnz(15, "root_total")
    p.send(1, 1, 14)                    # RESULT(result + 1) to the parent
    p.halt()
    p.label("root_total")
    p.mov(4, 14)                        # "<n> actors"
    p.label("wait")
    p.halt()
    return p.assemble()
