// pmc_codec.hip -- single translation unit for libpmc_codec.so (gfx950).
// One TU keeps the __constant__ tables in one module without relocatable device code.
#include "pmc_deflate.hip"
#include "pmc_deflate_small.hip"
#include "pmc_deflate_split.hip"
#include "pmc_deflate_large.hip"
#include "pmc_inflate.hip"
#include "pmc_inflate_lane.hip"
#include "pmc_inflate_rec.hip"
#include "pmc_misc.hip"
#include "pmc_capi.hip"
#include "pmc_store.hip"
#include "pmc_group.hip"
