"""Generate juicefs_amd/csrc/jfsx_sbox_bs.h: the bitsliced AES S-box as v_bitop3 ops.

Source circuit: J. Boyar and R. Peralta, "A depth-16 circuit for the AES S-box"
(2012), 34 AND + 94 XOR/XNOR gates (top linear layer T1..T27, non-linear middle
M1..M63, bottom linear layer L0..L29, outputs S0..S7; U0 / S0 are the most
significant bits).  The generator

  * turns the four XNOR outputs into XOR and leaves the complement (0x63) to the
    caller's per-output mask (which also carries the folded round key),
  * appends "S_i ^= mask_i" to every output,
  * maps the network onto three-input functions (cut enumeration with an
    area-flow cover and exact-area recovery, logic duplicated where that saves
    ops), so each emitted op is one v_bitop3_b32 (truth table =
    f(0xF0, 0xCC, 0xAA), src0 most significant),
  * verifies the fused program against the S-box table for all 256 inputs and
    every mask (bit-exact) before writing the header.

Run: python3 scripts/gen_sbox.py  (writes the header, prints the op count)."""
import os
import random
import sys

CIRCUIT = """
T1 = U0 + U3
T2 = U0 + U5
T3 = U0 + U6
T4 = U3 + U5
T5 = U4 + U6
T6 = T1 + T5
T7 = U1 + U2
T8 = U7 + T6
T9 = U7 + T7
T10 = T6 + T7
T11 = U1 + U5
T12 = U2 + U5
T13 = T3 + T4
T14 = T6 + T11
T15 = T5 + T11
T16 = T5 + T12
T17 = T9 + T16
T18 = U3 + U7
T19 = T7 + T18
T20 = T1 + T19
T21 = U6 + U7
T22 = T7 + T21
T23 = T2 + T22
T24 = T2 + T10
T25 = T20 + T17
T26 = T3 + T16
T27 = T1 + T12
M1 = T13 x T6
M2 = T23 x T8
M3 = T14 + M1
M4 = T19 x U7
M5 = M4 + M1
M6 = T3 x T16
M7 = T22 x T9
M8 = T26 + M6
M9 = T20 x T17
M10 = M9 + M6
M11 = T1 x T15
M12 = T4 x T27
M13 = M12 + M11
M14 = T2 x T10
M15 = M14 + M11
M16 = M3 + M2
M17 = M5 + T24
M18 = M8 + M7
M19 = M10 + M15
M20 = M16 + M13
M21 = M17 + M15
M22 = M18 + M13
M23 = M19 + T25
M24 = M22 + M23
M25 = M22 x M20
M26 = M21 + M25
M27 = M20 + M21
M28 = M23 + M25
M29 = M28 x M27
M30 = M26 x M24
M31 = M20 x M23
M32 = M27 x M31
M33 = M27 + M25
M34 = M21 x M22
M35 = M24 x M34
M36 = M24 + M25
M37 = M21 + M29
M38 = M32 + M33
M39 = M23 + M30
M40 = M35 + M36
M41 = M38 + M40
M42 = M37 + M39
M43 = M37 + M38
M44 = M39 + M40
M45 = M42 + M41
M46 = M44 x T6
M47 = M40 x T8
M48 = M39 x U7
M49 = M43 x T16
M50 = M38 x T9
M51 = M37 x T17
M52 = M42 x T15
M53 = M45 x T27
M54 = M41 x T10
M55 = M44 x T13
M56 = M40 x T23
M57 = M39 x T19
M58 = M43 x T3
M59 = M38 x T22
M60 = M37 x T20
M61 = M42 x T1
M62 = M45 x T4
M63 = M41 x T2
L0 = M61 + M62
L1 = M50 + M56
L2 = M46 + M48
L3 = M47 + M55
L4 = M54 + M58
L5 = M49 + M61
L6 = M62 + L5
L7 = M46 + L3
L8 = M51 + M59
L9 = M52 + M53
L10 = M53 + L4
L11 = M60 + L2
L12 = M48 + M51
L13 = M50 + L0
L14 = M52 + M61
L15 = M55 + L1
L16 = M56 + L0
L17 = M57 + L1
L18 = M58 + L8
L19 = M63 + L4
L20 = L0 + L1
L21 = L1 + L7
L22 = L3 + L12
L23 = L18 + L2
L24 = L15 + L9
L25 = L6 + L10
L26 = L7 + L9
L27 = L8 + L10
L28 = L11 + L14
L29 = L11 + L17
S0 = L6 + L24
S1 = L16 # L26
S2 = L19 # L28
S3 = L6 + L21
S4 = L20 + L22
S5 = L25 + L29
S6 = L13 # L27
S7 = L6 # L23
"""

A, B, C = 0xF0, 0xCC, 0xAA


def sbox_table():
    def mul(a, b):
        r = 0
        while b:
            if b & 1:
                r ^= a
            a = ((a << 1) ^ 0x11B) if a & 0x80 else a << 1
            b >>= 1
        return r
    inv = [0] * 256
    for a in range(1, 256):
        for b in range(1, 256):
            if mul(a, b) == 1:
                inv[a] = b
                break
    out = []
    for a in range(256):
        x = inv[a]
        y = x
        for i in range(1, 5):
            y ^= ((x << i) | (x >> (8 - i))) & 0xFF
        out.append(y ^ 0x63)
    return out


def parse():
    gates = []
    for line in CIRCUIT.strip().splitlines():
        lhs, rhs = [s.strip() for s in line.split("=")]
        if " x " in rhs:
            a, b = [s.strip() for s in rhs.split(" x ")]
            op = "and"
        elif "#" in rhs:
            a, b = [s.strip() for s in rhs.split("#")]
            op = "xor"  # complement carried by the caller's mask (0x63)
        else:
            a, b = [s.strip() for s in rhs.split("+")]
            op = "xor"
        gates.append((lhs, op, [a, b]))
    for i in range(8):  # S_i ^= mask_i
        gates.append(("O%d" % i, "xor", ["S%d" % i, "m%d" % i]))
    return gates


def fuse(gates, seed=0):
    """3-input technology mapping of the 2-input gate network (cut enumeration,
    area-flow cover, then exact-area recovery; logic may be duplicated across
    cuts).  Returns [(name, leaves, truth table)] in topological order."""
    nodes = {name: (op, ins) for name, op, ins in gates}
    order = [name for name, _, _ in gates]
    pis = {x for _, _, ins in gates for x in ins if x not in nodes}
    outs = [n for n in order if n.startswith("O")]
    fanout = {}
    for _, _, ins in gates:
        for x in ins:
            fanout[x] = fanout.get(x, 0) + 1
    cuts = {p: [frozenset([p])] for p in pis}
    for n in order:
        a, b = nodes[n][1]
        cs = {frozenset([n])}
        for ca in cuts[a]:
            for cb in cuts[b]:
                u = ca | cb
                if len(u) <= 3:
                    cs.add(u)
        cuts[n] = sorted(cs, key=lambda c: (len(c), sorted(c)))
        if seed:
            random.Random(seed * 1000003 + len(cuts)).shuffle(cuts[n])

    def real(n):
        return [c for c in cuts[n] if c != frozenset([n])]

    # area flow
    af, best = {}, {}
    for n in order:
        v_best = None
        for c in real(n):
            v = 1.0 + sum(0 if l in pis else af[l] / max(1, fanout.get(l, 1)) for l in c)
            if v_best is None or v < v_best:
                v_best, best[n] = v, c
        af[n] = v_best

    def used():
        need, stack = set(), list(outs)
        while stack:
            n = stack.pop()
            if n in need or n in pis:
                continue
            need.add(n)
            stack.extend(l for l in best[n] if l not in pis)
        return need

    def exact_area(c, refs):
        cnt, stack, seen = 1, [l for l in c if l not in pis], set()
        while stack:
            l = stack.pop()
            if l in seen:
                continue
            seen.add(l)
            if refs.get(l, 0) == 0:
                cnt += 1
                stack.extend(x for x in best[l] if x not in pis)
        return cnt

    for _ in range(20):
        need = used()
        refs = {}
        for n in need:
            for l in best[n]:
                if l not in pis:
                    refs[l] = refs.get(l, 0) + 1
        changed = False
        for n in order:
            if n not in need:
                continue
            cur = best[n]
            for l in cur:
                if l not in pis:
                    refs[l] -= 1
            v_best, c_best = None, None
            for c in real(n):
                v = exact_area(c, refs)
                if v_best is None or v < v_best:
                    v_best, c_best = v, c
            for l in c_best:
                if l not in pis:
                    refs[l] = refs.get(l, 0) + 1
            if c_best != cur:
                best[n], changed = c_best, True
        if not changed:
            break

    def evaluate(n, env, cache):
        if n in env:
            return env[n]
        if n not in cache:
            op, (a, b) = nodes[n]
            va, vb = evaluate(a, env, cache), evaluate(b, env, cache)
            cache[n] = (va & vb) if op == "and" else (va ^ vb)
        return cache[n]

    need = used()
    emit = []
    for n in order:
        if n in need:
            lv = sorted(best[n])
            emit.append((n, lv, evaluate(n, dict(zip(lv, (A, B, C))), {}) & 0xFF))
    return emit


def verify(emit):
    sb = sbox_table()
    for mask in (0x00, 0x63, 0xFF, 0x5A):
        for x in range(256):
            env = {"U%d" % i: -((x >> (7 - i)) & 1) & 0xFFFFFFFF for i in range(8)}
            for i in range(8):
                env["m%d" % i] = -(((mask ^ 0x63) >> (7 - i)) & 1) & 0xFFFFFFFF
            for name, lv, tt in emit:
                vals = [env[l] for l in lv] + [0] * (3 - len(lv))
                r = 0
                for bit in range(8):
                    if (tt >> bit) & 1:
                        a = vals[0] if bit & 4 else ~vals[0]
                        b = vals[1] if bit & 2 else ~vals[1]
                        c = vals[2] if bit & 1 else ~vals[2]
                        r |= a & b & c
                env[name] = r & 0xFFFFFFFF
            y = 0
            for i in range(8):
                y |= (env["O%d" % i] & 1) << (7 - i)
            assert y == sb[x] ^ mask, (x, mask)


def main():
    # tie-breaking among equal-area cuts changes the cover: keep the smallest
    emit = min((fuse(parse(), seed) for seed in range(400)), key=len)
    verify(emit)
    lines = [
        "// jfsx_sbox_bs.h -- GENERATED by scripts/gen_sbox.py; do not edit.",
        "// Bitsliced AES S-box (Boyar-Peralta depth-16 circuit, 128 gates) mapped onto",
        "// %d three-input ops.  In: U0..U7 (U0 = bit 7 of the byte), masks m0..m7" % len(emit),
        "// (m_i = all-ones where output bit 7-i is complemented: round key ^ 0x63).",
        "// Out: O0..O7 = S(U) ^ mask.  BS3(a, b, c, tt) is one v_bitop3_b32.",
        "#define JFSX_SBOX_BS(U0, U1, U2, U3, U4, U5, U6, U7, m0, m1, m2, m3, m4, m5, m6, m7, O0, O1, O2, O3, O4, O5, O6, O7) \\",
        "    do { \\",
    ]
    outs = {"O%d" % i for i in range(8)}
    for name, lv, tt in emit:
        args = list(lv) + ["0u"] * (3 - len(lv))
        dst = name if name in outs else "const uint32_t " + name
        lines.append("        %s = BS3(%s, %s, %s, 0x%02x); \\" % (dst, args[0], args[1], args[2], tt))
    lines.append("    } while (0)")
    lines.append("")
    # two S-boxes with their gates interleaved (independent chains back to back)
    lines.append("// Two S-boxes, gate by gate interleaved: suffix a / b.")
    pa = ["U%d" % i for i in range(8)] + ["m%d" % i for i in range(8)] + ["O%d" % i for i in range(8)]
    lines.append("#define JFSX_SBOX_BS2(" + ", ".join([x + "a" for x in pa] + [x + "b" for x in pa]) + ") \\")
    lines.append("    do { \\")
    for name, lv, tt in emit:
        for suf in "ab":
            args = [l + suf for l in lv] + ["0u"] * (3 - len(lv))
            dst = name + suf if name in outs else "const uint32_t " + name + suf
            lines.append("        %s = BS3(%s, %s, %s, 0x%02x); \\" % (dst, args[0], args[1], args[2], tt))
    lines.append("    } while (0)")
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "juicefs_amd", "csrc", "jfsx_sbox_bs.h")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("ops", len(emit), "->", os.path.normpath(path))


if __name__ == "__main__":
    sys.exit(main())
