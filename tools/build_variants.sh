#!/bin/bash
# Build tuning variants of libyafaray4.so into libyafaray_amd/variants/<name>.so
#   tools/build_variants.sh name1 "EXTRA flags" name2 "EXTRA flags" ...
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p $R/libyafaray_amd/variants
while [ $# -ge 2 ]; do
	make -s -C $R/libyafaray_amd/csrc OUT=$R/libyafaray_amd/variants/$1.so OBJ=$R/libyafaray_amd/build/v_$1 EXTRA="$2" >/dev/null
	echo "built $1: $2"
	shift 2
done
