module github.com/simple-pbft-amd/pbftv

go 1.19
