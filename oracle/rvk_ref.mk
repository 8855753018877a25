# oracle/_ref/librvk_ref.a: the reference's scalar-crypto helpers
# (src/arch/riscv/rvk.hh, a self-contained header) compiled where they lie
# under /root/reference through the C entry point oracle/rvk_ref.cc.  Test
# infrastructure only: the oracle links it for Zkn/Zks; nothing under
# shrewd_amd/ does.
REF_SRC ?= /root/reference/src
CXX ?= g++

_ref/librvk_ref.a: rvk_ref.cc $(REF_SRC)/arch/riscv/rvk.hh
	@mkdir -p _ref/obj
	$(CXX) -O2 -fPIC -std=c++17 -w -I$(REF_SRC) -c -o _ref/obj/rvk_ref.o rvk_ref.cc
	rm -f $@
	ar rcs $@ _ref/obj/rvk_ref.o
