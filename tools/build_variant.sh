#!/bin/bash
# Build an A/B variant of the product library from the working tree:
#   tools/build_variant.sh NAME 'sed-expr' [file]  -> build/ab/NAME/liblsbm_crc32c.so
# (the sed expression is applied to lsbm_amd/csrc/<file>, default crc32c_types.h)
set -e
cd "$(dirname "$0")/.."
name=$1; expr=$2; file=${3:-crc32c_types.h}
tmp=/tmp/lsbm_var_$name
rm -rf $tmp; mkdir -p $tmp/lsbm_amd $tmp/build
cp -r include $tmp/; cp -r lsbm_amd/csrc $tmp/lsbm_amd/
sed -i "$expr" $tmp/lsbm_amd/csrc/$file
grep -q . $tmp/lsbm_amd/csrc/$file
make -C $tmp/lsbm_amd/csrc -j8 >/dev/null
mkdir -p build/ab/$name
cp $tmp/lsbm_amd/liblsbm_crc32c.so build/ab/$name/
echo "build/ab/$name/liblsbm_crc32c.so"
