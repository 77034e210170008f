#!/bin/bash
# usage: tools/dump_kernel_asm.sh <file.hip> <mangled-kernel-name-regex> [extra hipcc flags]
# Writes the kernel's gfx950 assembly to /tmp/asm/kernel.s and prints instruction counts.
set -e
src=$1
pat=$2
shift 2
mkdir -p /tmp/asm
cd /tmp/asm
rm -f ./*.s
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -I/root/repo/include \
  -I/root/repo/gsdr_amd/csrc "$@" -c "/root/repo/$src" -o k.o -save-temps 2>/dev/null
S=$(ls ./*gfx950.s)
name=$(grep -oE "^_Z[A-Za-z0-9_]*:" "$S" | grep -E "$pat" | head -1 | tr -d ':')
awk -v n="$name:" 'index($0, n) == 1 {p = 1} p {print} p && /s_endpgm/ {exit}' "$S" > /tmp/asm/kernel.s
echo "$name -> /tmp/asm/kernel.s ($(wc -l < /tmp/asm/kernel.s) lines)"
for p in v_pk_fma_f32 v_fmac_f32 v_fma_f32 ds_read_b128 ds_read_b64 ds_write_b128 s_buffer_load global_load s_waitcnt s_barrier; do
  printf "%-16s %s\n" "$p" "$(grep -c "$p" /tmp/asm/kernel.s || true)"
done
