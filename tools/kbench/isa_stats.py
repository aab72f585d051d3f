"""Per-kernel ISA statistics of a device-only assembly listing of bp_decode.hip:
instruction count, VGPRs, ds_bpermute count, scratch use.
  hipcc ... --cuda-device-only -S -o k.s qec_ldpc_amd/csrc/bp_decode.hip
  python tools/kbench/isa_stats.py k.s [name-substring]"""
import re
import sys


def main():
    s = open(sys.argv[1]).read()
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for m in re.finditer(r"^(_Z\S*bp_decode_kernel\S*):", s, re.M):
        name = m.group(1)
        if sub not in name:
            continue
        body = s[m.end():s.index(".Lfunc_end", m.end())]
        meta = s[s.index(".amdhsa_kernel " + name):]
        vg = re.search(r"\.amdhsa_next_free_vgpr (\d+)", meta).group(1)
        n = len(re.findall(r"^\s+[vsdgb][a-z_0-9]+ ", body, re.M))
        short = re.sub(r"GeneratedShifts<.*", "", name)
        print("%-60s %-8s instrs %6d vgpr %4s bperm %4d scratch %d" % (
            name[:60], "split" if name.endswith("Lb1EEEvNS_6BpArgsE") else "", n, vg, body.count("ds_bpermute"),
            body.count("scratch_")))


if __name__ == "__main__":
    main()
