#!/bin/bash
# instruction histogram of inner loop number $3 (default 1) of kernel $2 in assembly file $1
awk -v k="$2" 'index($0, k) == 1 && /:/ {on=1} on {print} on && /s_endpgm/ {exit}' "$1" > /tmp/_k.s
n=${3:-1}
L=$(grep -n "Loop Header" /tmp/_k.s | sed -n "${n}p" | cut -d: -f1)
E=$(awk -v l="$L" 'NR>l && /s_cbranch_scc1|s_cbranch_vccnz|s_cbranch_scc0/ {print NR; exit}' /tmp/_k.s)
echo "loop lines $L-$E"
sed -n "${L},${E}p" /tmp/_k.s | grep -v "^\s*;" | grep -v "^\." | awk '{print $1}' | sort | uniq -c | sort -rn
