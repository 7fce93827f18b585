#!/usr/bin/env python3
"""Extract the fixtures a reference test script writes with heredocs (`cat > NAME << EOF ...
EOF`) into tests/golden/data/<dest>/ -- input VCFs and expected outputs, as data (test
infrastructure; run here, where /root/reference exists).

    python tests/golden/extract_sh_fixtures.py /root/reference/tests/test_dosage_calculator.sh ref_dosage
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def extract(script, dest):
    text = open(script).read()
    out = os.path.join(HERE, "data", dest)
    os.makedirs(out, exist_ok=True)
    n = 0
    for m in re.finditer(r"^cat > ([\w.]+) << '?EOF'?\n(.*?)^EOF$", text, re.M | re.S):
        name, body = m.group(1), m.group(2)
        if "$" in body or "`" in body:  # generated content (loops, variables): not a fixture
            continue
        with open(os.path.join(out, name), "w") as f:
            f.write(body)
        n += 1
    return n


if __name__ == "__main__":
    print(extract(sys.argv[1], sys.argv[2]), "files")
