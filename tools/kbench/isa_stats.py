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
        rx = re.match(r"_ZN3qec16bp_decode_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d)", name)
        tune = re.search(r"(SeqSynTune|ListTune|MinReg|Phase|RuntimeShifts)", name)
        mode = re.search(r"ELi(\d)EEEvNS_6BpArgsE$", name)
        stopn = {"0": "ref", "1": "fixed", "2": "syn"}[rx.group(4)] if rx else "?"
        sc = re.search(r"ScratchSize: (\d+)", meta)
        print("J%s K%s L%s %-5s mode %s %-13s instrs %6d vgpr %4s bperm %4d scratch-instrs %d scratch %s B" % (
            rx.group(1) if rx else "?", rx.group(2) if rx else "?", rx.group(3) if rx else "?", stopn,
            mode.group(1) if mode else "?", tune.group(1) if tune else "", n, vg, body.count("ds_bpermute"),
            body.count("scratch_"), sc.group(1) if sc else "?"))


if __name__ == "__main__":
    main()
