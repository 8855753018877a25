# oracle/_ref/libsoftfloat_ref.a: the reference's own SoftFloat (gem5
# ext/softfloat: SoftFloat 3 with the RISC-V specialization) compiled from its
# sources where they lie under /root/reference, with the flags of its
# SConscript (SOFTFLOAT_FAST_INT64) and per-thread state (-DTHREAD_LOCAL=__thread,
# the hook softfloat.h provides), for the oracle's F/D/Zfh arithmetic and the
# pinning tests of the device port.  Test infrastructure only: nothing under
# shrewd_amd/ links it.  The file list is the SConscript's SoftfloatFile() list
# up to its `else:` branch (use_fast_int64 is on, so that branch is not built).
REF_SF ?= /root/reference/ext/softfloat
CC ?= gcc
SF_SRCS := $(addprefix $(REF_SF)/,$(shell sed -n "/^else:/q; s/^ *SoftfloatFile('\(.*\)')/\1/p" $(REF_SF)/SConscript))
SF_OBJS := $(patsubst $(REF_SF)/%.c,_ref/obj/%.o,$(SF_SRCS))
SF_CFLAGS := -O2 -fPIC -w -DSOFTFLOAT_FAST_INT64 -DTHREAD_LOCAL=__thread -I$(REF_SF)

# a static archive, as the SConscript builds it (sf_env.Library): the oracle
# pulls in the members it calls
_ref/libsoftfloat_ref.a: $(SF_OBJS)
	rm -f $@
	ar rcs $@ $(SF_OBJS)

_ref/obj/%.o: $(REF_SF)/%.c
	@mkdir -p _ref/obj
	$(CC) $(SF_CFLAGS) -c -o $@ $<
