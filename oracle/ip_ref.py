"""Oracle: CPU restatement of the interest-point text files (.ip.txt).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  Follows
/root/reference/src/main/java/spim/fiji/spimdata/interestpoints/InterestPointList.java:
saveInterestPoints (:66-100: header "id\\tx\\ty\\tz", then id \\t x \\t y \\t z per point,
PrintWriter.println) and loadInterestPoints (:178-220: skip to the "id" header, split on
tab).  The doubles are printed by java.lang.Double.toString, restated here from its
specification (JDK 19+): the shortest decimal that uniquely distinguishes the value
(Python's repr digits), plain notation for 1e-3 <= |d| < 1e7 with at least one
fractional digit, else "d.dddE<exp>".  PARITY UNPINNED against a JVM (none in this
container); JDK <= 18 may print a longer digit string for a few values.
"""
from __future__ import annotations

import math


def java_double_to_string(d: float) -> str:
    d = float(d)
    if math.isnan(d):
        return "NaN"
    if math.isinf(d):
        return "Infinity" if d > 0 else "-Infinity"
    if d == 0.0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    sign = "-" if d < 0 else ""
    a = abs(d)
    mant, exp = f"{abs(d):.17e}".split("e")          # placeholder, replaced below
    r = repr(abs(d))                                    # shortest round-trip digits
    if "e" in r:
        m, e = r.split("e")
        e = int(e)
    else:
        m, e = r, 0
    if "." in m:
        ip, fp = m.split(".")
    else:
        ip, fp = m, ""
    digits = (ip + fp).lstrip("0")
    # decimal exponent of the first significant digit
    if ip.strip("0"):
        e1 = e + len(ip.lstrip("0")) - 1
    else:
        e1 = e - (len(fp) - len(fp.lstrip("0"))) - 1
    digits = digits.rstrip("0") or "0"
    del mant, exp
    if len(digits) == 1:
        # JDK 19+ spec: when the shortest decimal has one digit, the decimals of length
        # 1 or 2 that round to d compete and the closest wins (Double.MIN_VALUE prints
        # "4.9E-324", not "5.0E-324")
        from decimal import Decimal
        two = f"{a:.1e}"
        if float(two) == a:
            one = Decimal(f"{digits}e{e1}")
            if abs(Decimal(two) - Decimal(a)) < abs(one - Decimal(a)):
                m2, e2 = two.split("e")
                digits, e1 = m2.replace(".", "").rstrip("0") or "0", int(e2)
    if 1e-3 <= a < 1e7:
        if e1 >= 0:
            ipart = digits[:e1 + 1].ljust(e1 + 1, "0")
            fpart = digits[e1 + 1:] or "0"
            return f"{sign}{ipart}.{fpart}"
        return f"{sign}0.{'0' * (-e1 - 1)}{digits}"
    return f"{sign}{digits[0]}.{digits[1:] or '0'}E{e1}"


def ip_txt(points, ids=None) -> str:
    """The file text saveInterestPoints writes for points [(x, y, z)]."""
    lines = ["id\tx\ty\tz"]
    for i, p in enumerate(points):
        pid = i if ids is None else ids[i]
        lines.append(f"{pid}\t" + "\t".join(java_double_to_string(c) for c in p[:3]))
    return "\n".join(lines) + "\n"
