"""Instruction mix of the MFMA main loop of each kernel in a hipcc -S output (dev tool).

usage: python tools/asm_loop_stats.py file.s [name-substring ...]
"""
import re
import sys


def kernels(text):
    for m in re.finditer(r"^(\S+):\s*(?:;.*)?$\n", text, re.M):
        name = m.group(1)
        if name.startswith(".") or name.startswith("_Z") is False:
            continue
        end = text.find(".Lfunc_end", m.end())  # a kernel can hold several s_endpgm
        yield name, text[m.end():end]


def loop_of(body):
    lines = body.splitlines()
    first = next((i for i, l in enumerate(lines) if "v_mfma" in l), None)
    if first is None:
        return None
    hdr = None
    for i in range(first, -1, -1):
        if "Loop Header" in lines[i]:
            hdr = i if lines[i].startswith(".LBB") else i - 1  # the comment may have its own line
            break
    if hdr is None:
        return None
    label = lines[hdr].split(":")[0]
    end = None
    for i in range(first, len(lines)):
        if re.search(r"s_c?branch\w*\s+" + re.escape(label) + r"(\s|$)", lines[i]):
            end = i
    return lines[hdr:end + 1] if end else None


def stats(loop):
    ins = [l.strip() for l in loop if l.strip() and not l.strip().startswith((".", ";"))]
    c = lambda p: sum(1 for l in ins if re.match(p, l))  # noqa: E731
    waits = [l for l in ins if l.startswith("s_waitcnt") and "vmcnt" in l]
    return dict(total=len(ins), mfma=c(r"v_mfma"), valu=c(r"v_") - c(r"v_mfma"), salu=c(r"s_"),
                bufld=c(r"buffer_load"), gld=c(r"global_load"), dsr=c(r"ds_read"), dsw=c(r"ds_write"),
                barrier=c(r"s_barrier"), vmwaits=" ".join(w.split()[-1] for w in waits))


if __name__ == "__main__":
    text = open(sys.argv[1]).read()
    subs = sys.argv[2:]
    for name, body in kernels(text):
        if subs and not any(s in name for s in subs):
            continue
        lp = loop_of(body)
        if lp:
            print(name[-60:], stats(lp))
