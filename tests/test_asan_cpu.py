"""The host C++ under AddressSanitizer + UBSan (`make -C boda-1_amd asan`; SURVEY §5's counterpart
of the reference's memcheck runs, doc/debug-culibs.txt:4-11), on the CPU: every GPU-free mode over
every committed input, then over deterministic mutations of them (truncations, byte flips, spliced
lines) -- the parsers of untrusted text (nda_digest.cc hex / binary decode, lexp.cc, op_desc.cc,
conv_pipe.cc's prototxt reader, wis_ana.cc) must either succeed or fail with their own error, never
with a sanitizer report."""
import glob
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "boda-1_amd")
BIN = os.path.join(PKG, "bin", "asan")
G = os.path.join(ROOT, "tests", "golden")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:exitcode=86:abort_on_error=0",
           UBSAN_OPTIONS="halt_on_error=1:exitcode=87:print_stacktrace=1")


@pytest.fixture(scope="module", autouse=True)
def asan_build():
    subprocess.run(["make", "-j8", "asan"], cwd=PKG, check=True, stdout=subprocess.DEVNULL)


ERR = (0, 1, 2, 3, 4)  # success, or the tool's own error exits (usage 2, rt_err 3, unsup_err 4)


def run(tool, *args, ok_codes=(0,)):
    p = subprocess.run([os.path.join(BIN, tool)] + list(args), env=ENV, capture_output=True, text=True, errors="replace", timeout=300)
    report = ("AddressSanitizer" in p.stderr or "runtime error:" in p.stderr or "LeakSanitizer" in p.stderr
              or p.returncode in (86, 87) or p.returncode < 0)
    assert not report, "%s %s: rc %d\n%s" % (tool, " ".join(args), p.returncode, p.stderr[-3000:])
    assert p.returncode in ok_codes, (tool, args, p.returncode, p.stderr[-2000:])
    return p


@pytest.mark.parametrize("wis", sorted(glob.glob(os.path.join(G, "wis", "*.wis"))), ids=os.path.basename)
def test_selftest_wisdom(wis):
    assert "selftest ok" in run("boda_hip_ops_prof", "--selftest-wisdom=" + wis).stdout


@pytest.mark.parametrize("ops", sorted(glob.glob(os.path.join(G, "ops", "*.txt"))), ids=os.path.basename)
def test_dump_ops_and_shards(ops):
    run("boda_hip_ops_prof", "--dump-ops=" + ops, ok_codes=ERR)
    for k in range(3):
        run("boda_hip_ops_prof", "--list-shard=%d/3" % k, "--ops-fn=" + ops, ok_codes=ERR)


@pytest.mark.parametrize("net", sorted(glob.glob(os.path.join(G, "nets", "*.prototxt"))), ids=os.path.basename)
def test_prototxt_plans(net):
    for extra in (["--plan"], ["--plan-json"], ["--plan", "--no-fold", "--no-inplace-concat", "--no-resadd"]):
        run("boda_hip_rtc_fwd", "--net", net, "--img", "20", *extra)


def test_wis_ana(tmp_path):
    out = tmp_path / "wa.csv"
    run("boda_hip_wis_ana", "--wisdom-in-fn=" + os.path.join(G, "wis", "conv-debug.wis"), "--csv-out-fn=" + str(out),
        ok_codes=ERR)


def mutations(data, seed, n):
    """n deterministic corruptions of a text file: truncations, byte flips, dropped / doubled lines."""
    rng = random.Random(seed)
    lines = data.split(b"\n")
    out = []
    for i in range(n):
        k = i % 4
        if k == 0:
            out.append(data[:rng.randrange(1, len(data))])
        elif k == 1:
            b = bytearray(data)
            for _ in range(rng.randrange(1, 8)):
                b[rng.randrange(len(b))] = rng.choice(b"()=,. x0123456789abcdef\n\t-+e\x00\xff")
            out.append(bytes(b))
        elif k == 2:
            j = rng.randrange(len(lines))
            out.append(b"\n".join(lines[:j] + lines[j + 1:]))
        else:
            j = rng.randrange(len(lines))
            l = lines[j]
            c = rng.randrange(len(l) + 1)
            out.append(b"\n".join(lines[:j] + [l[:c] + l[c // 2:]] + lines[j + 1:]))
    return out


def test_mutated_inputs(tmp_path):
    cases = [("conv-debug.wis", "wis", lambda f: ("boda_hip_ops_prof", "--selftest-wisdom=" + f)),
             ("sgemm-gen5.wis", "wis", lambda f: ("boda_hip_ops_prof", "--selftest-wisdom=" + f)),
             ("conv-ops-debug.txt", "ops", lambda f: ("boda_hip_ops_prof", "--dump-ops=" + f)),
             ("op_sigs_full.txt", "ops", lambda f: ("boda_hip_ops_prof", "--dump-ops=" + f)),
             ("googlenet_conv.prototxt", "nets", lambda f: ("boda_hip_rtc_fwd", "--net", f, "--plan")),
             ("resnet-50.prototxt", "nets", lambda f: ("boda_hip_rtc_fwd", "--net", f, "--plan"))]
    n = 0
    for fn, sub, cmd in cases:
        data = open(os.path.join(G, sub, fn), "rb").read()
        if len(data) > 200000:  # the big wisdom files: their head is the parser's whole state machine
            data = data[:200000]
        for i, m in enumerate(mutations(data, sum(fn.encode()), 48)):
            p = tmp_path / ("m%d_%s" % (i, fn))
            p.write_bytes(m)
            run(*cmd(str(p)), ok_codes=ERR)
            n += 1
    assert n == 48 * len(cases)
