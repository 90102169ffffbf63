VARIANTS="pb qnoinl qinl qnoinl pb" bash tools/ablate.sh
