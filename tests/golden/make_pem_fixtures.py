"""Extract the PEM key fixtures that the reference's own tests hold
(pkg/object/encrypt_test.go:33-67: keyInPKCS8, an encrypted PKCS#8 key with
passphrase "12345678", and pemWithoutPass, a PKCS#1 key) into
tests/golden/pem_fixtures.json.  Data only: run here, where /root/reference
exists; the JSON travels, the reference does not."""
import json
import os
import re

SRC = "/root/reference/pkg/object/encrypt_test.go"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pem_fixtures.json")


def main():
    text = open(SRC).read()
    fx = {}
    for name in ("keyInPKCS8", "pemWithoutPass"):
        m = re.search(r"var %s = `(.*?)`" % name, text, re.S)
        fx[name] = m.group(1)
    fx["source"] = "pkg/object/encrypt_test.go:33-67 (TestParsePKCS8 :69-78, TestParsePemWithoutPassword :80-89)"
    with open(OUT, "w") as f:
        json.dump(fx, f, indent=1)


if __name__ == "__main__":
    main()
