"""The kernels skip a transformation whose trigger bytes do not occur in the
value (csrc/gi_program.h transform_triggers / byte_summary).  Check that
claim against the oracle's transformations: on random values built only from
bytes outside a transformation's trigger set, the oracle returns the value
unchanged."""
import random

import pytest

import gpuinspect
from oracle import coraza

# TCode (csrc/gi_program.h) -> oracle transformation name
CODES = {1: "lowercase", 2: "urldecode", 3: "urldecodeuni", 4: "htmlentitydecode", 5: "removenulls",
         6: "replacenulls", 7: "removewhitespace", 8: "compresswhitespace", 9: "replacecomments", 10: "cmdline",
         11: "length", 12: "trim", 13: "trimleft", 14: "trimright", 15: "normalizepath", 16: "normalizepathwin",
         17: "jsdecode", 18: "utf8tounicode", 19: "base64decode", 20: "base64decodeext", 21: "base64encode",
         22: "hexdecode", 23: "hexencode", 24: "sha1", 25: "md5", 26: "urlencode", 27: "cssdecode",
         28: "escapeseqdecode", 29: "removecommentschar"}


@pytest.mark.parametrize("code", sorted(CODES))
def test_untriggered_transform_is_identity(code):
    trig, summ = gpuinspect.selftest_triggers()
    if trig[code] == 0xFFFFFFFF:  # always applied (transform_identity never holds): nothing to check
        return
    quiet = [b for b in range(256) if not (summ[b] & trig[code])]
    assert quiet, code
    fn = coraza.TRANSFORM_FNS[CODES[code]]
    rnd = random.Random(code)
    for _ in range(3000):
        n = rnd.randrange(0, 40)
        v = bytes(rnd.choice(quiet) for _ in range(n))
        assert fn(v) == v, (CODES[code], v)


def test_summary_bits_cover_trigger_bytes():
    trig, summ = gpuinspect.selftest_triggers()
    # spot checks of the byte classes the triggers are built from
    for ch, t in ((b"%", 2), (b"+", 3), (b"&", 4), (b"A", 1), (b"\x80", 18), (b"\x00", 5), (b" ", 7), (b"/", 15),
                  (b"\\", 17), (b".", 15), (b"'", 10), (b"^", 10), (b";", 10)):
        assert summ[ch[0]] & trig[t], (ch, CODES[t])
