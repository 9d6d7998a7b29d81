#!/bin/bash
# Tuning builds of the MFMA edge kernels: libpfsgnn_<name>.so = the normal
# objects with pfsgnn_mfma.o and pfsgnn_sliced.o rebuilt under extra -D flags
# (pfsgnn_mfma.hip as ONE object, MF_PART 0: MF_SRC_KEEP is the header's
# default 1 for every kernel unless the flags set it);
# select one at run time with PFSGNN_LIB_VARIANT=<name> (pfsgnn/native.py).
#   bash tools/variants.sh name1 "-DMF_DEPTH_BWD=3" name2 "-DCOL_CH=16" ...
set -e
cd "$(dirname "$0")/../pfs-neural-net_amd"
make -j8 >/dev/null
objs=$(ls build/*.o | grep -v -e 'pfsgnn_mfma\.o' -e pfsgnn_mfma_ebwd -e pfsgnn_sliced.o -e var_ -e pfsgnn_loss_exact.o)
flags=$(make -s -f - print <<'MK'
include Makefile
print:
	@echo $(MFMA_FLAGS)
MK
)
pids=()
while [ $# -gt 0 ]; do
  name=$1; def=$2; shift 2
  ( /opt/rocm/bin/hipcc $flags $def -c csrc/pfsgnn_mfma.hip -o build/var_$name.o &&
    /opt/rocm/bin/hipcc $flags $def -c csrc/pfsgnn_sliced.hip -o build/var_sl_$name.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o pfsgnn/libpfsgnn_$name.so $objs build/var_$name.o build/var_sl_$name.o &&
    echo "built libpfsgnn_$name.so ($def)" ) &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
