"""Random libsvm text generators for parity tests (emulator and GPU).

uniform_libsvm() draws from the grammar the single-pass kernel handles
(svm_fast.h: digitchar runs, blanks, ':' and newlines, including the odd
corners of ParsePair -- runs of signs/dots/exponents, stray colons after a
newline, CR/LF mixes, tabs, label:weight, missing values, very long runs and
gaps).  With violate=True it also injects the constructs that must send the
input to the exact kernels ('#', "qid:", letters, dangling "x:", "a:b:c").
"""
import numpy as np

_NUM = ["0", "1", "7", "42", "007", "+3", "-0", "0.5", ".5", "5.", "1e-3", "-2.5E+7", "3.4028235e38",
        "1e39", "1e-45", "123456789012345678901234", "0.123456789012345678901234", "+", "-", ".",
        "e", "E5", "1e", "1.5e-", "--1", "+-2", "9" * 30]


def _num(rng):
    if rng.random() < 0.6:
        return "%.9g" % rng.random() if rng.random() < 0.7 else str(int(rng.integers(0, 10 ** 6)))
    return _NUM[int(rng.integers(0, len(_NUM)))]


def _idx(rng):
    if rng.random() < 0.85:
        return str(int(rng.integers(0, 5000)))
    return ["0", "4294967297", "+12", "3.7", "1e3", "00", "18446744073709551617"][int(rng.integers(0, 7))]


def _blank(rng):
    r = rng.random()
    if r < 0.8:
        return " "
    if r < 0.9:
        return "\t"
    return " " * int(rng.integers(2, 90))


def _line(rng, maxfeat, violate):
    parts = []
    if rng.random() < 0.1:
        parts.append(_blank(rng))
    if rng.random() < 0.05:
        parts.append(":")  # colon before the label: skipped by ParsePair
    parts.append(_num(rng))
    if rng.random() < 0.15:
        parts.append(rng.choice([":", " :", ": ", " : "]) + _num(rng))
    for _ in range(int(rng.integers(0, maxfeat + 1))):
        parts.append(_blank(rng))
        parts.append(_idx(rng))
        if rng.random() < 0.93:
            parts.append(rng.choice([":", ":", ":", " :", ": ", ":\t"]) + _num(rng))
    if violate and rng.random() < 0.2:
        parts.append(rng.choice([" # c", " qid:3", " 3:", " 1:2:3", "x", " 2:nan", " 5:inf", ":"]))
    if rng.random() < 0.1:
        parts.append(_blank(rng))
    return "".join(parts)


def uniform_libsvm(rng, nlines, maxfeat=40, violate=False):
    out = []
    for _ in range(nlines):
        r = rng.random()
        if r < 0.04:
            out.append("")  # blank line
        elif r < 0.06:
            out.append(_blank(rng))
        else:
            out.append(_line(rng, maxfeat, violate))
    seps = ["\n"] * 12 + ["\r\n", "\r", "\n\n"]
    text = "".join(line + seps[int(rng.integers(0, len(seps)))] for line in out)
    if rng.random() < 0.3:
        text = text.rstrip("\r\n")  # no trailing newline
    return text.encode("latin-1")


def qid_libsvm(rng, nlines, maxfeat=40, violate=False, mixed=False, long_head=False):
    """libsvm ranking rows, "<label>[:<weight>] qid:<n> <idx>:<val> ...", in the
    fast grammar (svm_fast.h qid_clean / qid_ok): the token after the label
    (any blanks) or after label:weight (spaces), 1-18 digits.  violate=True
    mixes in the forms the reference reads differently (a tab after the
    weight, "qid: 5", "qid:5.5", a second token, a token among the features,
    19 digits, stray letters); mixed=True leaves some rows without a qid;
    long_head=True makes some line heads longer than 64 bytes (long labels and
    weights, long blank runs before the token)."""
    out = []
    for _ in range(nlines):
        if rng.random() < 0.03:
            out.append("")
            continue
        parts = [_num(rng) if rng.random() < 0.3 else str(int(rng.integers(0, 5)))]
        wt = rng.random() < 0.25
        if wt:
            parts.append(rng.choice([":", " :", ": "]) + _num(rng))
        q = str(int(rng.integers(0, 10 ** int(rng.integers(1, 19)))))
        sep = rng.choice([" ", "  ", " ", ""] if wt else [" ", "\t", "  ", " \t", ""])
        if long_head and rng.random() < 0.4:
            k = int(rng.integers(30, 90))
            pick = int(rng.integers(0, 3))
            if pick == 0:
                sep = " " * k if wt else rng.choice([" " * k, "\t" * (k // 3) + " "])
            elif pick == 1:
                parts[0] = parts[0] + "0" * k if "." in parts[0] else parts[0] + "." + "1" * k
            elif wt:
                parts[-1] = parts[-1] + "5" * k if "." in parts[-1] else parts[-1] + ".0" + "7" * k
        tok = sep + "qid:" + q
        if violate and rng.random() < 0.15:
            tok = rng.choice(["\tqid:" + q if wt else " qid: " + q, " qid:5.5", " qid:-3", " qid:", " qid:5:3",
                              " QID:1", " qidd:1", " qid:1 qid:2", " qid:" + "9" * 19, " iqd:4", " q"])
        if not (mixed and rng.random() < 0.1):
            parts.append(tok)
        for j in range(int(rng.integers(0, maxfeat + 1))):
            parts.append(_blank(rng) + _idx(rng) + ":" + _num(rng))
            if violate and rng.random() < 0.01:
                parts.append(" qid:7")
        out.append("".join(parts))
    seps = ["\n"] * 12 + ["\r\n", "\r"]
    text = "".join(line + seps[int(rng.integers(0, len(seps)))] for line in out)
    return text.encode("latin-1")


def comment_libsvm(rng, nlines, maxfeat=30, long_frac=0.0, violate=False, qid=False, line_comments=False):
    """libsvm rows with '#' comments where IgnoreCommentAndBlank reads them
    (libsvm_parser.h:67-83): whole comment lines, a header at the start, and
    trailing comments after a label, an index, a value or a qid, with or
    without blanks before the '#'; comment text is any printable byte but a
    newline (letters, digits, ':', "qid:", more '#').  long_frac: share of
    comments longer than a tile's pre-halo (64 B).  violate=True adds forms
    the reference reads otherwise ('#' after a ':' or "qid:", stray letters).
    line_comments=True adds '#' lines after the first, which the reference
    does not read as comments (ParseBlock's lines begin at the previous '\\n',
    which IgnoreCommentAndBlank does not skip: their digits become rows)."""
    alphabet = "abcdefghijklmnopqrstuvwxyz ABCXYZ0123456789:.+-eE#\t qid:qid !?,;=_/"

    def ctext():
        n = int(rng.integers(70, 400)) if rng.random() < long_frac else int(rng.integers(0, 50))
        return "".join(alphabet[int(rng.integers(0, len(alphabet)))] for _ in range(n)).replace("\\t", "\t")

    out = []
    if rng.random() < 0.5:
        out.append(rng.choice(["#", " #", "\t# "]) + ctext())
    for _ in range(nlines):
        r = rng.random()
        if line_comments and r < 0.08:
            out.append(rng.choice(["", " ", "\t"]) + "#" + ctext())
            continue
        parts = [_num(rng) if rng.random() < 0.3 else str(int(rng.integers(0, 5)))]
        if rng.random() < 0.2:
            parts.append(":" + _num(rng))
        if qid:
            parts.append(" qid:" + str(int(rng.integers(0, 1000))))
        for j in range(int(rng.integers(0, maxfeat + 1))):
            parts.append(_blank(rng) + _idx(rng) + (":" + _num(rng) if rng.random() < 0.9 else ""))
        if rng.random() < 0.5:
            parts.append(rng.choice(["", " ", "  ", "\t", " \t"]) + "#" + ctext())
        if violate and rng.random() < 0.1:
            parts.append(rng.choice([" 3:#x", " 3: # y", " qid:#1", " a#", " #:", " 5 :#"]))
        out.append("".join(parts))
    seps = ["\n"] * 12 + ["\r\n", "\r"]
    text = "".join(line + seps[int(rng.integers(0, len(seps)))] for line in out)
    return text.encode("latin-1")


def dense_libsvm(rng, nbytes, style):
    """libsvm text with the shortest runs the grammar allows, so a 16 KiB tile
    holds several thousand runs (the fast kernel's run lists then take
    several passes): 'pairs' "1:2 3:4 ...", 'weights' "l:w i:v ...",
    'labels' one-digit label-only lines, 'mixed' all of them."""
    out, n = [], 0
    while n < nbytes:
        st = style if style != "mixed" else ("pairs", "weights", "labels")[int(rng.integers(0, 3))]
        d = lambda: str(int(rng.integers(0, 10)))
        if st == "labels":
            line = d()
        elif st == "weights":
            line = d() + ":" + d() + "".join(" %s:%s" % (d(), d()) for _ in range(int(rng.integers(1, 40))))
        else:
            line = d() + "".join(" %s:%s" % (d(), d()) for _ in range(int(rng.integers(1, 60))))
        out.append(line)
        n += len(line) + 1
    return ("\n".join(out) + "\n").encode("latin-1")


def dense_libfm(rng, nbytes):
    """libfm rows of one-digit triples ("l f:i:v f:i:v ..."): several thousand
    runs per 16 KiB tile, so the libfm run lists (indices, fields, values) take
    several passes."""
    out, n = [], 0
    while n < nbytes:
        d = lambda: str(int(rng.integers(0, 10)))
        line = d() + (":" + d() if rng.random() < 0.2 else "") + "".join(
            " %s:%s:%s" % (d(), d(), d()) for _ in range(int(rng.integers(1, 50))))
        out.append(line)
        n += len(line) + 1
    return ("\n".join(out) + "\n").encode("latin-1")


def _csv_field(rng):
    r = rng.random()
    if r < 0.08:
        return ""  # empty field: the column advances, nothing is pushed
    if r < 0.75:
        return "%.9g" % (rng.random() * 2 - 1)
    return _NUM[int(rng.integers(0, len(_NUM)))]


def uniform_csv(rng, nlines, maxcols=40, delim=",", violate=False):
    """CSV in the grammar the single-pass CSV kernel handles (csv_fast.h):
    number characters, the delimiter and newlines -- empty fields, trailing
    delimiters, blank lines, CR/LF mixes, odd numbers.  violate=True also
    injects bytes that send the input to the exact kernels."""
    out = []
    for _ in range(nlines):
        r = rng.random()
        if r < 0.04:
            out.append("")
            continue
        ncol = int(rng.integers(1, maxcols + 1))
        line = delim.join(_csv_field(rng) for _ in range(ncol))
        if rng.random() < 0.05:
            line += delim
        if violate and rng.random() < 0.2:
            line += rng.choice([" ", "\t1", "nan", "x", "\xef\xbb\xbf"])
        out.append(line)
    seps = ["\n"] * 12 + ["\r\n", "\r", "\n\n"]
    text = "".join(line + seps[int(rng.integers(0, len(seps)))] for line in out)
    if rng.random() < 0.3:
        text = text.rstrip("\r\n")
    return text.encode("latin-1")


_JUNK = ["abc", "x1", "?", "#c", '"q"', "col_7", "hello world", "3.5kg", "12abc", "-x", "+", "-", ".", "e",
         "e5", "1e", "0x1A", "W", "(null)", "$9", "_", "a.b", "1/2", "2021-01-02", "feature", "F", "-f", "name",
         "index", "id", "int", "NAME", "-nam", "in", "n", "i", "f5", "fin"]


def junk_csv(rng, nlines, maxcols=30, delim=",", header=True, violate=False):
    """CSV with text fields (csv_fast.h csv_junk_byte): a header row of column
    names, text columns and words among the numbers, numbers followed by text
    ("3.5kg"): ParseFloat consumes nothing of a field that starts with text
    (no value, the column advances) and stops at text after a number
    (csv_parser.h:99-127); an 'f' at a field start is its suffix (the value 0);
    "nan" / "inf" / "Infinity" (any case, after a sign or blanks) are values,
    text after blanks a 0, bytes >= 0x80 junk, and a UTF-8 BOM at a row start
    is skipped (IgnoreUTF8BOM).  violate=True adds one field of ParseFloat's
    "NaN(chars)" form (strtonum.h:157-165) -- closed (a NaN), or not (the
    reference's fatal "Invalid NAN literal") -- which the single pass takes
    since round 6."""
    ncol = int(rng.integers(1, maxcols + 1))
    out = []
    if header:
        out.append(delim.join("c%d_%s" % (j, "xyz"[j % 3]) for j in range(ncol)))
    for _ in range(nlines):
        if rng.random() < 0.03:
            out.append("")
            continue
        fields = []
        for j in range(ncol if rng.random() < 0.9 else int(rng.integers(1, ncol + 1))):
            r = rng.random()
            if r < 0.15:
                v = _JUNK[int(rng.integers(0, len(_JUNK)))]
            elif r < 0.2:
                v = ""
            else:
                v = _csv_field(rng)
            if rng.random() < 0.03:
                v = rng.choice(["nan", "inf", "Infinity", "-inf", "+NAN", "info", " abc", "\xef\xbb\xbf1",
                                "\t?", " nan", "  -Inf", "nAn", "-nan", "\xe9t\xe9", "in", "na", "infin", "infinit",
                                "INFINITY", "-Infinity7", "infx", "nana"])
            fields.append(v.replace(delim, ";") if delim != ";" else v.replace(delim, ":"))
        row = delim.join(fields)
        bom = "\xef\xbb\xbf" if rng.random() < 0.05 and row[:1] not in ("", "\r") else ""  # (a BOM ending its line: exact)
        out.append(bom + row)
    if violate and len(out) > 1:
        k = int(rng.integers(1, len(out)))
        form = ["NaN(1)", "nan(x_y)", "-nan(ab)", " nan(q)", "NaN(1", "nan(a-b)", "+NAN()"][int(rng.integers(0, 7))]
        out[k] = form + delim + out[k]
    seps = ["\n"] * 12 + ["\r\n", "\r"]
    text = "".join(line + seps[int(rng.integers(0, len(seps)))] for line in out)
    return text.encode("latin-1")


def dense_csv(rng, nbytes, delim=",", wide=False):
    """CSV of one-digit fields (some empty): up to 8k tokens per 16 KiB tile,
    so the CSV token lists (csv_fast.h kPassTokens) take several passes; rows
    that span tiles carry their column in from the look-back.  wide=True adds
    a row of more than 2^17 columns (past the list's column field: the exact
    kernels)."""
    out, n = [], 0
    while n < nbytes:
        ncol = int(rng.integers(1, 4000 if rng.random() < 0.3 else 60))
        if wide and not out:
            ncol = (1 << 17) + 300
        f = rng.integers(0, 11, size=ncol)
        line = delim.join("" if v == 10 else str(v) for v in f)
        out.append(line)
        n += len(line) + 1
    seps = ["\n"] * 12 + ["\r\n", "\n\n"]
    return "".join(line + seps[int(rng.integers(0, len(seps)))] for line in out).encode("latin-1")


def random_cuts(rng, data, nmax=8, anywhere=False):
    """Chunk offsets: after a newline (as an InputSplit cuts), or, with
    anywhere=True, at arbitrary bytes (the C-ABI allows any chunking)."""
    n = len(data)
    if n == 0:
        return [0]
    if anywhere:
        cand = list(range(1, n))
    else:
        a = np.frombuffer(data, dtype=np.uint8)
        cand = (np.flatnonzero((a == 10) | (a == 13)) + 1).tolist()
        cand = [c for c in cand if c < n]
    k = int(rng.integers(0, min(nmax, len(cand)) + 1)) if cand else 0
    cuts = sorted(set(rng.choice(cand, size=k, replace=False).tolist())) if k else []
    return [0] + cuts + [n]


def libfm_rows(rng, rows, width, weights=False):
    """Synthetic libfm text: 'label[:w] field:index:value ...' per line
    (libfm_parser.h:67-144), ids 1-based and increasing, values %.9g."""
    out = []
    for _ in range(rows):
        lab = "%d" % int(rng.integers(0, 2))
        if weights:
            lab += ":%.6g" % float(rng.random())
        ids = np.cumsum(rng.integers(1, 9, size=width))
        flds = rng.integers(1, 40, size=width)
        vals = rng.random(width).astype(np.float32)
        out.append(lab + " " + " ".join("%d:%d:%.9g" % (f, i, v) for f, i, v in zip(flds, ids, vals)))
    return ("\n".join(out) + "\n").encode()


def labeled_csv(rng, nlines, ncols, label_col, delim=",", defects=0.0, weight_col=-1):
    """CSV with a label column: every row holds ncols non-empty numeric fields
    (the single-pass kernel's label form) unless a defect is injected with
    probability `defects`: an empty label field, a short row, a one-field row,
    empty value fields or a trailing delimiter."""
    out = []
    for _ in range(nlines):
        fields = ["%.9g" % v for v in (rng.random(ncols).astype(np.float32) * 2 - 1)]
        fields[min(label_col, ncols - 1)] = str(int(rng.integers(0, 2)))
        if rng.random() < defects:
            kind = int(rng.integers(0, 5))
            if kind == 0:
                fields[min(weight_col if weight_col >= 0 and rng.random() < 0.5 else label_col, ncols - 1)] = ""
            elif kind == 1:
                fields = fields[:int(rng.integers(1, max(2, label_col + 1)))]
            elif kind == 2:
                fields = fields[:1]
            elif kind == 3:
                fields[int(rng.integers(0, ncols))] = ""
            else:
                fields.append("")
        out.append(delim.join(fields))
    return ("\n".join(out) + "\n").encode()


def uniform_libfm(rng, nlines, maxtrip=20, violate=False):
    """libfm lines in the single-pass kernel's grammar (digitchars, blanks, ':'
    and newlines): label[:weight], field:index[:value] groups, dropped lone
    fields, pairs without values, blank lines; violate=True also injects
    structures that leave it ("a:b:c:d", "l:w:x", dangling "f:", signs)."""
    lines = []
    for _ in range(nlines):
        if rng.random() < 0.05:
            lines.append(" " * int(rng.integers(0, 3)))
            continue
        head = str(int(rng.integers(0, 3)))
        if rng.random() < 0.2:
            head += ":%.4g" % float(rng.random())
        parts = [head]
        for _ in range(int(rng.integers(0, maxtrip + 1))):
            f, i = int(rng.integers(0, 50)), int(rng.integers(0, 3000))
            r = rng.random()
            if r < 0.1:
                parts.append("%d" % f)  # lone field: dropped (r = 1)
            elif r < 0.25:
                parts.append("%d:%d" % (f, i))  # no value (r = 2)
            else:
                parts.append("%d:%d:%.9g" % (f, i, float(rng.random()) * (10 ** int(rng.integers(-2, 4)))))
        if violate and rng.random() < 0.3:
            parts.append(["1:2:3:4", "-3:4:5", "7:", "+2:3:4", "5:-6:1"][int(rng.integers(0, 5))])
        sep = " " * int(rng.integers(1, 3)) if rng.random() < 0.2 else " "
        lines.append(sep.join(parts))
    ends = ["\n"] * 10 + ["\r\n", "\n\n"]
    text = "".join(l + ends[int(rng.integers(0, len(ends)))] for l in lines)
    return text.encode()


_INTS = ["0", "7", "-3", "+12", "007", "019", "08", "-0", "2147483648", "-2147483649", "99999999",
         "123456789", "9223372036854775808", "-9223372036854775809", "1e5", "2.5", "-.5", ".5", "+", "-",
         "e", "00", "0.0", "-0.123"]


def blank_csv(rng, nlines, maxcols=30, delim=",", ints=False, violate=False):
    """CSV with blanks around the values (", " separators, padded and
    blank-only fields): ParseFloat / strtoll skip the blanks before a value
    and the reference skips anything after it up to the delimiter
    (csv_parser.h:99-127).  ints=True draws integer-looking fields (octal,
    overflow, signs, fractions).  violate=True adds a blank-only last field (the
    decoder would read on into the next line: the exact kernels)."""
    out = []
    for _ in range(nlines):
        if rng.random() < 0.03:
            out.append(" " * int(rng.integers(0, 3)) if violate else "")
            continue
        fields = []
        for _ in range(int(rng.integers(1, maxcols + 1))):
            r = rng.random()
            if r < 0.06:
                v = ""
            elif r < 0.12:
                v = " " * int(rng.integers(1, 4))  # blank-only field
            elif ints:
                v = _INTS[int(rng.integers(0, len(_INTS)))] if rng.random() < 0.4 else str(int(rng.integers(-10 ** 6, 10 ** 6)))
            else:
                v = _csv_field(rng)
            if v.strip():
                v = " " * int(rng.integers(0, 3) if rng.random() < 0.7 else 0) + v
                if rng.random() < 0.2:
                    v += rng.choice([" ", "  ", "\t", " 9"])
            fields.append(v)
        if not fields[-1].strip() and not violate:
            fields[-1] = ""  # a blank-only last field reads on into the next line
        line = delim.join(fields)
        if violate and rng.random() < 0.15:
            line += delim + " "
        out.append(line)
    seps = ["\n"] * 10 + ["\r\n", "\n\n"]
    return "".join(line + seps[int(rng.integers(0, len(seps)))] for line in out).encode("latin-1")


DIRTY_LINES = ["# synth libsvm shard", "# hdr", "#!", "junk", "@@@", "7 abc 3:4", "x 1:2 3:4", "5 1:0.5 zz 2:7",
               "1 2:3 # a comment x", "   hdr  ", "8 qid-less 4:1", "3 1:2 ~ 5:6", "0 1:0.25 2:", "2 !1:3",
               "9 3:nan 4:1", "4 1:inf", "6 NaN(1):2", "1 2:0.5 3:-inf"]


def dirty_libsvm(rng, nbytes, rate=0.002, long_frac=0.0, near_tile_end=False, eol=b"\n"):
    """Uniform-grammar libsvm rows (about nbytes) with lines holding bytes
    outside the grammar -- "# header" lines of the next file after InputSplit's
    '\n' between files (input_split_base.cc:204-210), words, stray symbols,
    inf / nan values -- at a share `rate` of the lines; long_frac: share of
    them longer than 256 bytes.  near_tile_end: put dirty lines across and
    near the 16 KiB single-pass tile ends.  eol: the line end ("\n", "\r\n"
    or a lone "\r" -- the reference ends a line at either byte,
    libsvm_parser.h:95)."""
    body = uniform_libsvm(rng, max(1, nbytes // 60), 12).replace(b"\r", b"\n")
    lines = body.split(b"\n")
    out = []
    pos = 0
    e = len(eol)
    for ln in lines:
        if rng.random() < rate:
            d = DIRTY_LINES[int(rng.integers(0, len(DIRTY_LINES)))].encode()
            if rng.random() < long_frac:
                d = d + b" " + b"1:2 " * int(rng.integers(70, 120))
            if rng.random() < 0.5:
                d = eol + d  # the empty line InputSplit leaves between files
            if near_tile_end:
                t_end = (pos // 16384 + 1) * 16384
                gap = t_end - pos - int(rng.integers(-40, 100))
                if 0 < gap < 400:
                    out.append(b"1" + b" " * max(0, gap - 1 - e))
                    pos += len(out[-1]) + e
            out.append(d)
            pos += len(d) + e
        out.append(ln)
        pos += len(ln) + e
    return eol.join(out) + eol


# Dirty tokens inside rows (round 6, svm_fast.h dirty_rewrite): words (with
# digitchar letters e/E and the qid letters q / i / d among them), symbols,
# bytes >= 0x80, a vertical tab, an unreachable '#' (behind a non-blank byte:
# no comment, libsvm_parser.h:67-83), a ':' behind a non-blank
# byte -- all of which ParsePair skips like blanks except where they stand
# between a run and its ':' (strtonum.h:683-687) -- and ParseFloat's inf /
# nan forms after a sign (strtonum.h:133-175).  (An unsigned "nan" value
# is skipped to the next run, "a:b:c" -- the exact kernels take that.)
ROW_TOKENS = [b"NA", b"null", b"did", b"x", b"~", b"@@", b"qi", b"dq", b"x#y", b"\x0b", b"\xc3\xa9t\xc3\xa9", b"!",
              b"n/a", b"q:"]
# tokens holding digitchar runs of their own (read as index-only ids: a block
# mixing them with valued pairs fails the reference's RowBlock CHECK,
# row_block.h:178 -- the tests then compare the failure)
RUN_TOKENS = [b"feature", b"note", b"Eq", b"id:4", b"x:3", b"x#5", b"(1)", b"idx=7"]
VALUE_TOKENS = [b"-inf", b"+nan", b"-Infinity", b"-nan(7)", b"+INF", b"-x", b"+", b"-n"]


def dirty_rows_libsvm(rng, nrows, width, rate=0.125, eol=b"\n", near_tile_end=False, runs=False):
    """libsvm rows of `width` pairs (ids increasing, "%.9g" values) where a
    share `rate` of the rows carries 1-3 dirty tokens: a word between pairs,
    an inf / nan value ("3:-inf") or label; with `runs`, also words holding
    digitchar runs and words glued to an index ("5x:0.3": index-only pairs).  No qid tokens, no dangling ':' and no
    "a:b:c" chains, so the single pass keeps every such input
    (dirty_rewrite) -- the tests check that it does and that the result is
    the reference's."""
    out = []
    pos = 0
    for r in range(nrows):
        ids = np.cumsum(rng.integers(1, 17, size=width)) - 1
        vals = rng.random(width).astype(np.float32)
        toks = [b"%d:%.9g" % (int(i), float(v)) for i, v in zip(ids, vals)]
        label = b"%d" % int(rng.integers(0, 2))
        if rng.random() < rate:
            for _ in range(int(rng.integers(1, 4))):
                kind = rng.random()
                j = int(rng.integers(0, width)) if width else 0
                pool = ROW_TOKENS + RUN_TOKENS if runs else ROW_TOKENS
                if kind < 0.45 or width == 0:
                    toks.insert(j, pool[int(rng.integers(0, len(pool)))])
                elif kind < 0.65 and runs:
                    t = pool[int(rng.integers(0, len(pool)))].split(b":")[0]
                    if b":" in toks[j]:  # (not a token inserted before)
                        toks[j] = b"%s%s:%s" % (toks[j].split(b":")[0], t, toks[j].split(b":")[1])
                elif kind < 0.95:
                    if b":" in toks[j]:
                        toks[j] = b"%s:%s" % (toks[j].split(b":")[0], VALUE_TOKENS[int(rng.integers(0, len(VALUE_TOKENS)))])
                else:
                    label = VALUE_TOKENS[int(rng.integers(0, len(VALUE_TOKENS)))]
        sep = b"\t" if rng.random() < 0.05 else b" "
        line = label + b"".join(sep + t for t in toks)
        if near_tile_end and rng.random() < 0.3:
            t_end = (pos // 16384 + 1) * 16384
            gap = t_end - pos - int(rng.integers(0, 64))
            if 0 < gap < 200:
                out.append(b"1" + b" " * max(0, gap - 1 - len(eol)))
                pos += len(out[-1]) + len(eol)
        out.append(line)
        pos += len(line) + len(eol)
    return eol.join(out) + eol


def long_row_libsvm(rng, form, row_kb=(34, 70)):
    """Short rows around one to three rows longer than four exact windows
    (> 32 KiB), so that at exact tile_bytes=4096 (three recorded windows per
    tile, args.h exact_rec_win) a row crosses tile ends past the count pass's
    records (libsvm_core.h: the write pass restores the role state and the
    pending token from rec_meta there).  form: "valued" (every pair has a
    value), "mid_pair" (the long row ends with an index and ':' missing),
    "dangling" (it ends with "idx:"), "long_head" (labels / values of up to
    ~300 digits, so tokens straddle window edges), "index_only" (no values)."""
    def tok(i):
        if form == "index_only":
            return "%d" % i
        if form == "long_head" and rng.random() < 0.02:
            return "%d:0.%s" % (i, "".join(rng.choice(list("0123456789"), int(rng.integers(50, 300)))))
        return "%d:%.6g" % (i, rng.random())
    def label():
        if form == "long_head" and rng.random() < 0.3:
            return "1." + "0" * int(rng.integers(100, 400)) + "1"
        return str(int(rng.integers(0, 2)))
    rows = []
    nlong = int(rng.integers(1, 4))
    where = sorted(rng.choice(np.arange(1, 40), nlong, replace=False).tolist())
    for r in range(40):
        if r in where:
            target = int(rng.integers(row_kb[0], row_kb[1])) << 10
            parts, n, i = [label()], 0, 0
            while n < target:
                i += int(rng.integers(1, 5))
                t = tok(i)
                parts.append(" " * int(rng.integers(1, 3)) + t)
                n += len(t) + 2
            if r == where[-1] and form == "mid_pair":
                parts.append(" %d" % (i + 1))
            elif r == where[-1] and form == "dangling":
                parts.append(" %d:" % (i + 1))
            rows.append("".join(parts))
        else:
            rows.append(" ".join([label()] + [tok(j) for j in range(int(rng.integers(0, 12)))]))
    pad = " " * int(rng.integers(0, 8192))  # moves the rows against the 4 KiB tiles and 8 KiB windows
    return (pad + "\n".join(rows) + "\n").encode()


def wide_row_csv(rng, row_kb=(34, 70)):
    """CSV rows with one to three rows wider than four exact windows (the
    CSV write pass recounts past its records, csv_core.h)."""
    rows = []
    ncol = None
    nlong = int(rng.integers(1, 4))
    where = set(rng.choice(np.arange(0, 30), nlong, replace=False).tolist())
    for r in range(30):
        if r in where:
            target = int(rng.integers(row_kb[0], row_kb[1])) << 10
            f, n = [], 0
            while n < target:
                x = "%.5g" % (rng.random() * 100) if rng.random() < 0.8 else ""
                f.append(x)
                n += len(x) + 1
            rows.append(",".join(f))
        else:
            rows.append(",".join("%.4g" % rng.random() for _ in range(int(rng.integers(1, 20)))))
    return ("\n".join(rows) + "\n").encode()
