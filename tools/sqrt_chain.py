#!/usr/bin/env python3
"""Product count of the decompression exponentiation y = a^((p+1)/4) on BLS12-381 (VERDICT r05
item 7): the shipped width-4 window (points.hpp fp_pow_sqrt29: 1 squaring + 7 products for the
odd table x..x^15, then the generated SQRT_* steps) against sliding windows of every width and
against lower bounds for any addition chain.

python tools/sqrt_chain.py
"""
import math

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
E = (P + 1) // 4


def sliding_window(e, w):
    """(squarings, products) of a left-to-right sliding window over odd digits < 2^w."""
    bits = bin(e)[2:]
    table = 1 + (1 << (w - 1)) - 1 if w > 1 else 0  # x^2 then x^3, x^5, ... x^(2^w - 1)
    sq = mul = 0
    i = 0
    first = True
    while i < len(bits):
        if bits[i] == "0":
            if not first:
                sq += 1
            i += 1
            continue
        j = min(len(bits), i + w)
        while bits[j - 1] == "0":
            j -= 1
        if first:
            first = False  # the first window's value is a table entry: no squaring, no product
        else:
            sq += j - i
            mul += 1
        i = j
    return sq, mul, table


def main():
    nb = E.bit_length()
    wt = bin(E).count("1")
    print("e = (p+1)/4: %d bits, Hamming weight %d" % (nb, wt))
    best = None
    for w in range(1, 10):
        sq, mul, tab = sliding_window(E, w)
        tot = sq + mul + tab
        print("sliding window w=%d: %d squarings + %d products + %d table = %d" % (w, sq, mul, tab, tot))
        if best is None or tot < best[0]:
            best = (tot, w)
    # any addition chain for e has length >= log2(e) + log2(v(e)) - 2.13 (Schoenhage)
    lb = math.log2(E) + math.log2(wt) - 2.13
    print("best sliding window: %d products (w=%d)" % best)
    print("Schoenhage lower bound for any addition chain: %.1f products" % lb)
    print("shipped (points.hpp, width 4): 461 products")


if __name__ == "__main__":
    main()
