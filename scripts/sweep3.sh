CONFIG=tridiag VARIANTS="kprefetch=0;kprefetch=2;kprefetch=4;nt_store=0;nt_load=0" bash scripts/variant_pmc.sh && \
CONFIG=vadv VARIANTS="kprefetch=0;kprefetch=2;kprefetch=4;nt_store=0" bash scripts/variant_pmc.sh && \
CONFIG=lap5 VARIANTS="prefetch=4;jchunk=8;jchunk=16;jchunk=32;prefetch=2;prefetch=6" bash scripts/variant_pmc.sh
