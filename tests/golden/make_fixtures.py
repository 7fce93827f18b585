#!/usr/bin/env python3
"""Write the crafted parity-trap fixtures into tests/golden/data/.

These are DATA, written deterministically by this script; the expected outputs for them
come from the reference binaries (tests/golden/make_golden.py).  Synthetic slices come
from build/bin/vcfx_synth (seeded, portable PRNG).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
DATA = os.path.join(HERE, "data")
REPO = os.path.dirname(os.path.dirname(HERE))

H = "##fileformat=VCFv4.2\n##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">\n"


def chrom_line(n):
    return "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT" + "".join(
        "\tS%d" % (i + 1) for i in range(n)) + "\n"


def w(name, text, mode="w"):
    with open(os.path.join(DATA, name), "wb") as f:
        f.write(text.encode("latin-1") if isinstance(text, str) else text)


def rec(chrom, pos, rid, ref, alt, qual, filt, info, fmt, samples):
    return "\t".join([chrom, str(pos), rid, ref, alt, qual, filt, info, fmt] + samples) + "\n"


def nonref_fixtures():
    """VCFX_nonref_filter traps: hom-ref spellings the two input modes
    judge differently ("000", "0", "/", polyploid, GT not first, missing subfields, empty
    samples, trailing tabs), FORMAT without GT, short lines, CRLF, empty lines, '#' lines
    between records and long all-hom-ref / one-non-ref records"""
    H = "##fileformat=VCFv4.2\n"
    body = H + "1\t1\tpre\tA\tC\t.\t.\t.\tGT\t0|0\n" + chrom_line(3)
    gts = ["0|0", "0/0", "000", "0", "00", "/", "|", "0/0/0", "0|0|0", "0/1", "1|0", "./.", ".", ".|0", "0|.",
           "0/0:5", "0:1", "", "0|0|1", "10/0", "0/00", "|0|", "0/0\t"]
    pos = 100
    for a in gts:
        for b in ("0|0", "0/1"):
            pos += 1
            body += rec("1", pos, "g%d" % pos, "A", "C", "50", "PASS", ".", "GT", [a, b, "0|0"])
    for fmt, samples in [("DP:GT", ["5:0|0", "7:0/0", "1:0|0"]), ("DP:GT", ["5:0|1", "7:0/0", "1:0|0"]),
                         ("DP:GT", ["5", "7:0/0", "1:0|0"]), ("GT:DP", ["0|0:5", "0/0", ":3"]),
                         ("DP", ["5", "6", "7"]), ("GTX:GT", ["1:0|0", "0:0|0", "0:0/0"]), ("", ["0|0", "0|0", "0|0"]),
                         ("GT:", ["0|0", "0|0", "0|0"]), (":GT", ["x:0|0", "y:0|0", ":0/0"]),
                         ("GT:GT", ["0|0:1|1", "0/0:1", "0|0"])]:
        pos += 1
        body += rec("1", pos, "f%d" % pos, "A", "C", "50", "PASS", ".", fmt, samples)
    body += "1\t%d\tshort\tA\tC\t50\tPASS\t.\tGT\n" % (pos + 1)
    body += "1\t%d\tshorter\tA\tC\t50\tPASS\n" % (pos + 2)
    body += "1\t%d\ttrail\tA\tC\t50\tPASS\t.\tGT\t0|0\t0|0\t\n" % (pos + 3)
    body += "1\t%d\tnine_tabs\tA\tC\t50\tPASS\t.\tGT\t\n" % (pos + 4)
    body += "\n#interleaved\n\n"
    long_ref = ["0|0"] * 3000
    body += rec("1", pos + 5, "allref", "A", "C", "50", "PASS", ".", "GT", long_ref)
    body += rec("1", pos + 6, "lastalt", "A", "C", "50", "PASS", ".", "GT", long_ref[:-1] + ["0|1"])
    body += rec("1", pos + 7, "firstalt", "A", "C", "50", "PASS", ".", "GT", ["1/1"] + long_ref[1:])
    body += rec("1", pos + 8, "missing", "A", "C", "50", "PASS", ".", "GT", long_ref[:1500] + ["./."] + long_ref[1501:])
    w(os.path.join("ref_nonref", "nonref_traps.vcf"), body)
    w(os.path.join("ref_nonref", "nonref_traps_crlf.vcf"), body.replace("\n", "\r\n"))


def main():
    os.makedirs(DATA, exist_ok=True)
    # --- genotype zoo: every GT token shape the AF/GQ/LD parsers branch on
    gts = ["0|1", "1/0", "./.", ".|1", "0/.", "2|1", "10/1", "0", "1", "0|1|2", "./1", "a/b",
           "00/1", ".", "0||1", "|1", "1|", "1/1", "0|0", "3/3", "01|1", ".a/1", "1 /0", "+1/0",
           "1/+0", "0/01", "11|11"]
    body = H + chrom_line(len(gts))
    body += rec("1", 100, "rsA", "A", "G", "50", "PASS", "AF=0.5", "GT", gts)
    body += rec("1", 200, "rsB", "C", "T", "60", "PASS", "AF=0.1", "GT:DP", [g + ":12" for g in gts])
    body += rec("1", 300, "rsC", "G", "A", "70", "q10", "DP=5", "DP:GT", ["7:" + g for g in gts])
    body += rec("1", 400, "rsD", "T", "C", ".", "PASS", ".", "DP", ["3"] * len(gts))
    body += rec("1", 500, ".", "A", "C,G", "80", "PASS", "AF=0.2,0.1", "GT:", [g + ":" for g in gts])
    body += rec("1", 600, "rsF", "A", "C", "80", "PASS", "AF=0.3", ":GT", [":" + g for g in gts])
    body += rec("1", 700, "rsG", "A", "C", "80", "PASS", "AF=0.3", "GT:AD:DP", [g + ":1,2:3" for g in gts])
    body += "1\t800\trsH\tA\tC\t90\tPASS\tAF=0.4\tGT\n"                 # FORMAT, no samples
    body += "1\t900\trsI\tA\tC\t90\tPASS\tAF=0.4\tGT\t\n"               # trailing tab
    body += "1\t1000\trsJ\tA\tC\t90\tPASS\tAF=0.4\tGT\t0|1\t\t1|1\n"    # empty sample
    body += "1\t1100\trsK\tA\tC\t90\tPASS\tAF=0.4\t\t0|1\t1|1\n"        # empty FORMAT
    body += "1\t1200\trsL\tA\tC\t90\tPASS\tAF=0.4\n"                    # 8 columns
    body += "1\t1300\trsM\tA\tC\n"                                      # 5 columns
    body += "\n"                                                       # empty line
    body += "##late_header=1\n"                                        # header after data
    body += "#CHROM_again\n"
    body += rec("2", 1400, "rsN", "A", "C", "1e2", "PASS", "AF=0x1A;DP= 7;FLAG", "GT", gts[:3])
    body += rec("2", 1500, "rsO", "A", "C", "inf", "PASS", "AF=nan;DP=1e400;FLAG", "GT", gts[3:6])
    body += rec("2", "0x10", "rsP", "A", "C", "-3.5", "LowQual", "AF=-0.0;DP=12abc", "GT", gts[6:9])
    body += rec("2", 1600, "rsQ", "A", "C", "  5", "PASS", "AF=.25;;DP=+3", "GT", ["1|1"] * 4)
    body += rec("2", 1700, "rsR", "A", "C", "99.9999999999999999999", "PASS", "AF=2.5e-1", "GT",
                ["0|1"] * 2 + ["1|0"] * 2 + ["0|0"])
    body += rec("2", 1800, "rsS", "A", "C", "", "PASS", "AF", "GT", ["0/1", "0|1", "1|1", "1/1"])
    w("edge_zoo.vcf", body)

    # --- rounding ties: 1 ALT of 32 alleles (=0.03125, a binary tie at 4 dp) and friends
    n = 16
    body = H + chrom_line(n)
    for k, alts in enumerate([1, 3, 5, 7, 9, 11, 13, 15, 16, 31, 32]):
        s = []
        left = alts
        for i in range(n):
            a0 = 1 if left > 0 else 0
            left -= a0
            a1 = 1 if left > 0 else 0
            left -= a1
            s.append("%d|%d" % (a0, a1))
        body += rec("3", 10 + k, "t%d" % k, "A", "T", "30", "PASS", "AF=%d" % alts, "GT", s)
    # 1/3 of 6, 2/3 etc; missing changes totals to create more ties (e.g. 1/16, 1/80)
    body += rec("3", 99, "t99", "A", "T", "30", "PASS", ".", "GT", ["1|0"] + ["0|0"] * 7 + ["./."] * 8)
    body += rec("3", 98, "t98", "A", "T", "30", "PASS", ".", "GT", ["1|0"] + ["0|0"] * 15)
    w("ties.vcf", body)

    # --- CRLF file (mmap strips \r, AF stdin does not)
    body = H + chrom_line(16)
    for k in range(5):
        s = ["%d|%d" % ((i + k) % 3 == 0, (i * k) % 5 == 0) for i in range(16)]
        body += rec("4", 100 + k, "c%d" % k, "A", "T", "30", "PASS" if k % 2 else "LowQual", "AF=0.%d" % k, "GT", s)
    w("crlf.vcf", body.replace("\n", "\r\n"))

    # --- data before #CHROM; no #CHROM; empty file; no trailing newline; header-only
    pre = H + rec("1", 5, "x", "A", "C", "9", "PASS", ".", "GT", ["0|1", "1|1"]) + chrom_line(2)
    pre += rec("1", 6, "y", "A", "C", "9", "PASS", ".", "GT", ["0|1", "1|1"])
    w("data_before_header.vcf", pre)
    w("no_chrom.vcf", H + rec("1", 5, "x", "A", "C", "9", "PASS", ".", "GT", ["0|1", "1|1"]))
    w("empty.vcf", "")
    w("no_trailing_newline.vcf", H + chrom_line(3) + rec("1", 5, "x", "A", "C", "9", "PASS", "AF=0.5", "GT",
                                                          ["0|1", "1|1", "0/0"]).rstrip("\n"))
    w("header_only.vcf", H + chrom_line(3))
    # more samples in records than in the header, and fewer
    body = H + chrom_line(3)
    body += rec("5", 10, "m1", "A", "C", "9", "PASS", ".", "GT", ["0|1", "1|1", "0|0", "1|1", "1|0"])
    body += rec("5", 20, "m2", "A", "C", "9", "PASS", ".", "GT", ["0|1"])
    body += rec("5", 30, "m3", "A", "C", "9", "PASS", ".", "GT", ["1|1", "0|1", "0|0"])
    body += rec("5", 40, "m4", "A", "C", "9", "PASS", ".", "GT", ["1|1", "1|1", "0|0"])
    w("ragged_samples.vcf", body)

    # --- gzip stdin for variant_counter (single member, and two concatenated members =
    #     BGZF-like: the reference counts only the first member)
    import gzip
    src = open(os.path.join(DATA, "ref", "variant_counter_normal.vcf"), "rb").read()
    w("vc_normal.vcf.gz", gzip.compress(src, mtime=0))
    half = src.index(b"\n", len(src) // 2) + 1
    w("vc_two_members.vcf.gz", gzip.compress(src[:half], mtime=0) + gzip.compress(src[half:], mtime=0))
    w("vc_corrupt.vcf.gz", gzip.compress(src, mtime=0)[:40] + b"garbage-garbage-garbage")

    # --- synthetic slices from the product's deterministic generator
    synth = os.path.join(REPO, "build", "bin", "vcfx_synth")
    if not os.path.exists(synth):
        sys.exit("build/bin/vcfx_synth missing: run make first")
    slices = [
        # name, records, samples, seed, info_mode, missing, hap, irregular, crlf
        ("synth_regular.vcf", 400, 2504, 7, 0, 0.0, 0, 0.0, 0),
        ("synth_annot.vcf", 300, 500, 11, 1, 0.0, 0, 0.0, 0),
        ("synth_missing.vcf", 300, 257, 13, 1, 0.02, 0, 0.0, 0),
        ("synth_irregular.vcf", 300, 301, 17, 1, 0.01, 0, 0.2, 0),
        ("synth_crlf.vcf", 120, 64, 19, 1, 0.01, 0, 0.1, 1),
        ("synth_ld.vcf", 160, 200, 23, 0, 0.01, 1, 0.0, 0),
    ]
    for name, m, ns, seed, info, miss, hap, irr, crlf in slices:
        subprocess.check_call([synth, os.path.join(DATA, name), str(m), str(ns), str(seed), str(info),
                               repr(miss), str(hap), repr(irr), str(crlf)])
    nonref_fixtures()
    print("fixtures written to", DATA)


if __name__ == "__main__":
    main()
