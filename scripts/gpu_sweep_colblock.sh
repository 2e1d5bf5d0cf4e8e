VC="col_bx=64;col_bx=256;col_order=1;col_bx=256,col_order=1;col_bx=128,col_order=1"
VCP="pointwise_plane=0;pointwise_plane=0,col_bx=256;pointwise_plane=0,col_order=1;pointwise_plane=0,col_bx=256,col_order=1;pointwise_plane=0,col_bx=128,col_order=1"
CONFIGS=copy VH="$VCP" bash scripts/gpu_sweep_plane.sh && CONFIGS="tridiag vadv" VH="$VC" bash scripts/gpu_sweep_plane.sh
